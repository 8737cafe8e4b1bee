#!/bin/bash
# Session check on a fresh box: the -m gpu suite, the C2 bench line and the
# sliding-window stream bench, each under its own limit; stops at the first
# failure. Outputs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --mode stream --steps 2 --warmup 1 > gpurun_out/bench_stream_sw.log 2>&1 || exit 3
