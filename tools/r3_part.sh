#!/bin/bash
# partitioned solve checks (gloo ranks sharing the GPU) + planning/full-batch timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/fb_timing.py C2 3 > gpurun_out/fb_timing_c2.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/fb_timing.py NS 2 > gpurun_out/fb_timing_ns.log 2>&1 || exit 2
timeout -k 10 560 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_partition.py -m gpu > gpurun_out/part_tests.log 2>&1 || exit 3
