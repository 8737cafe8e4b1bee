#!/bin/bash
# Bench lines of the round (C2 with the CPU baseline, NS, the stream modes,
# batched refinement) and the refinement kernel-trace profile; outputs under
# gpurun_out/bench/. Each step under its own limit; stops at the first failure.
set -o pipefail
o=gpurun_out/bench; mkdir -p $o
timeout -k 10 300 python -u bench.py > $o/bench_c2.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config NS --no-cpu-baseline > $o/bench_ns.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --mode stream --steps 2 --warmup 1 > $o/bench_stream_sw.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --mode stream --full-batch --steps 2 --warmup 1 > $o/bench_stream_fb.log 2>&1 || exit 4
timeout -k 10 300 python -u bench.py --mode refine --steps 3 --warmup 1 --cpu-seconds 10 > $o/bench_refine.log 2>&1 || exit 5
bash tools/prof_run.sh $o/prof_refine bench.py --mode refine --steps 2 --no-cpu-baseline > $o/prof_refine.txt 2>&1 || exit 6
