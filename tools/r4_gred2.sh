#!/bin/bash
# Reduced gather: large classes dispatched first (default) against smallest
# first (DYNOHIP_GRED_ORDER=small), NS and C2 kernel stats; bits against the
# round's previous build (variants/old).
set -o pipefail
o=gpurun_out/r4g2
mkdir -p $o
timeout -k 10 300 python -u tools/ab_bits.py run $o/new.npz C1 C2 NS > $o/ab_new.log 2>&1 || exit 1
python tools/ab_bits.py cmp gpurun_out/r4g/old.npz $o/new.npz > $o/ab_cmp.log 2>&1
bash tools/prof_run.sh $o/prof_ns bench.py --config NS --steps 2 --no-cpu-baseline > $o/prof_ns.txt 2>&1 || exit 2
DYNOHIP_GRED_ORDER=small bash tools/prof_run.sh $o/prof_ns_small bench.py --config NS --steps 2 --no-cpu-baseline > $o/prof_ns_small.txt 2>&1 || exit 3
bash tools/prof_run.sh $o/prof_c2 bench.py --steps 3 --no-cpu-baseline > $o/prof_c2.txt 2>&1 || exit 4
DYNOHIP_GRED_ORDER=small bash tools/prof_run.sh $o/prof_c2_small bench.py --steps 3 --no-cpu-baseline > $o/prof_c2_small.txt 2>&1 || exit 5
timeout -k 10 300 python -u bench.py --config NS --no-cpu-baseline > $o/bench_ns.log 2>&1 || exit 6
