#!/bin/bash
# Stream-mode measurements at the current build: the sliding-window bench
# line (3 replays) and a kernel-trace (with stats) of one replay, each under
# its own limit. Outputs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --mode stream --steps 3 --warmup 1 > gpurun_out/bench_stream_sw.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stream -o run --output-format csv -- python -u bench.py --mode stream --steps 1 --warmup 1 > gpurun_out/prof_stream.log 2>&1 || exit 2
