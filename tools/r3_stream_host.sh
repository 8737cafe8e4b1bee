#!/bin/bash
# stream mode: per-window planning/upload breakdown, stream bench, full-batch call timing
set -o pipefail
mkdir -p gpurun_out
DYNOHIP_PLAN_TIMING=1 timeout -k 10 300 python -u bench.py --mode stream --steps 1 --warmup 0 > gpurun_out/sh_stream_timing.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --mode stream --steps 3 --warmup 1 > gpurun_out/sh_stream.log 2>&1 || exit 2
timeout -k 10 200 python -u tools/fb_timing.py C2 4 > gpurun_out/sh_fb_c2.log 2>&1 || exit 3
