#!/bin/bash
# full-batch call breakdown at C2 (plan / upload / values / destroy), stream bench, then the GPU suite
set -o pipefail
mkdir -p gpurun_out
DYNOHIP_PLAN_TIMING=1 timeout -k 10 200 python -u tools/fb_timing.py C2 6 > gpurun_out/fb_c2_upload.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/fb_timing.py C2 6 > gpurun_out/fb_c2.log 2>&1 || exit 2
timeout -k 10 200 python -u tools/fb_timing.py NS 3 > gpurun_out/fb_ns.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --mode stream --steps 3 --warmup 1 > gpurun_out/stream.log 2>&1 || exit 4
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 5
