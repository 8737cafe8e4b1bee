#!/bin/bash
# Reduced gather: gradient blocks dispatched first (DYNOHIP_GRED_GRAD_FIRST=0:
# after the band); bits against the round's previous build (variants/old);
# kernel stats; the round's bench lines (C2 with the CPU baseline, NS, stream).
set -o pipefail
o=gpurun_out/r4g6
mkdir -p $o
DYNOSAM_AMD_LIB_DIR=variants/old timeout -k 10 300 python -u tools/ab_bits.py run $o/old.npz C1 C2 NS > $o/ab_old.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_bits.py run $o/new.npz C1 C2 NS > $o/ab_new.log 2>&1 || exit 2
python tools/ab_bits.py cmp $o/old.npz $o/new.npz > $o/ab_cmp.log 2>&1
bash tools/prof_run.sh $o/prof_ns bench.py --config NS --steps 2 --no-cpu-baseline > $o/prof_ns.txt 2>&1 || exit 3
DYNOHIP_GRED_GRAD_FIRST=0 bash tools/prof_run.sh $o/prof_ns_gl bench.py --config NS --steps 2 --no-cpu-baseline > $o/prof_ns_gl.txt 2>&1 || exit 4
bash tools/prof_run.sh $o/prof_c2 bench.py --steps 3 --no-cpu-baseline > $o/prof_c2.txt 2>&1 || exit 5
DYNOHIP_GRED_GRAD_FIRST=0 bash tools/prof_run.sh $o/prof_c2_gl bench.py --steps 3 --no-cpu-baseline > $o/prof_c2_gl.txt 2>&1 || exit 6
bash tools/prof_run.sh $o/prof_stream bench.py --mode stream --steps 1 --warmup 0 > $o/prof_stream.txt 2>&1 || exit 7
timeout -k 10 400 python -u bench.py > $o/bench_c2.log 2>&1 || exit 8
timeout -k 10 300 python -u bench.py --config NS > $o/bench_ns.log 2>&1 || exit 9
timeout -k 10 300 python -u bench.py --mode stream --steps 2 --warmup 1 > $o/bench_stream_sw.log 2>&1 || exit 10
