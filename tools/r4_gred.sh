#!/bin/bash
# Reduced gather in lane classes: A/B bits against the previous build
# (variants/old), kernel stats of C2 and NS with each build, bench lines.
set -o pipefail
o=gpurun_out/r4g
mkdir -p $o
DYNOSAM_AMD_LIB_DIR=variants/old timeout -k 10 300 python -u tools/ab_bits.py run $o/old.npz C1 C2 NS > $o/ab_old.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_bits.py run $o/new.npz C1 C2 NS > $o/ab_new.log 2>&1 || exit 2
python tools/ab_bits.py cmp $o/old.npz $o/new.npz > $o/ab_cmp.log 2>&1
bash tools/prof_run.sh $o/prof_c2 bench.py --steps 3 --no-cpu-baseline > $o/prof_c2.txt 2>&1 || exit 3
bash tools/prof_run.sh $o/prof_ns bench.py --config NS --steps 2 --no-cpu-baseline > $o/prof_ns.txt 2>&1 || exit 4
DYNOSAM_AMD_LIB_DIR=variants/old bash tools/prof_run.sh $o/prof_ns_old bench.py --config NS --steps 2 --no-cpu-baseline > $o/prof_ns_old.txt 2>&1 || exit 5
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $o/bench_c2.log 2>&1 || exit 6
timeout -k 10 300 python -u bench.py --config NS --no-cpu-baseline > $o/bench_ns.log 2>&1 || exit 7
DYNOSAM_AMD_LIB_DIR=variants/pipe3 bash tools/prof_run.sh $o/prof_ns_pipe3 bench.py --config NS --steps 2 --no-cpu-baseline > $o/prof_ns_pipe3.txt 2>&1 || exit 8
DYNOSAM_AMD_LIB_DIR=variants/pipe3 timeout -k 10 300 python -u tools/ab_bits.py run $o/pipe3.npz C1 C2 NS > $o/ab_pipe3.log 2>&1 || exit 9
python tools/ab_bits.py cmp $o/new.npz $o/pipe3.npz > $o/ab_cmp_pipe3.log 2>&1
