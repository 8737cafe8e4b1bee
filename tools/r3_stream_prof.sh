#!/bin/bash
# fresh-handle vs persistent full-batch call breakdown, and a kernel trace of
# the sliding-window stream replay (bench.py --mode stream)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/fb_timing.py C2 4 > gpurun_out/fb_timing_c2.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_stream -o run --output-format csv -- python -u bench.py --mode stream --steps 1 --warmup 1 > gpurun_out/prof_stream.log 2>&1 || exit 2
