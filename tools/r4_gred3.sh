#!/bin/bash
# Reduced gather: lone-group partial blocks added directly (kAddBlock), bits
# against the round's previous build (variants/old), NS and C2 kernel stats.
set -o pipefail
o=gpurun_out/r4g3
mkdir -p $o
DYNOSAM_AMD_LIB_DIR=variants/old timeout -k 10 300 python -u tools/ab_bits.py run $o/old.npz C1 C2 NS > $o/ab_old.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_bits.py run $o/new.npz C1 C2 NS > $o/ab_new.log 2>&1 || exit 2
python tools/ab_bits.py cmp $o/old.npz $o/new.npz > $o/ab_cmp.log 2>&1
bash tools/prof_run.sh $o/prof_ns bench.py --config NS --steps 2 --no-cpu-baseline > $o/prof_ns.txt 2>&1 || exit 3
bash tools/prof_run.sh $o/prof_c2 bench.py --steps 3 --no-cpu-baseline > $o/prof_c2.txt 2>&1 || exit 4
bash tools/prof_run.sh $o/prof_stream bench.py --mode stream --steps 1 --warmup 0 > $o/prof_stream.txt 2>&1 || exit 5
timeout -k 10 300 python -u bench.py --config NS --no-cpu-baseline > $o/bench_ns.log 2>&1 || exit 6
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $o/bench_c2.log 2>&1 || exit 7
