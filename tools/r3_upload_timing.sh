#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
DYNOHIP_PLAN_TIMING=1 timeout -k 10 200 python -u tools/fb_timing.py C2 4 > gpurun_out/fb_c2_upload.log 2>&1 || exit 1
