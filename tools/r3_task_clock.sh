#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
DYNOSAM_AMD_LIB_DIR=variants/tclk timeout -k 10 200 python tools/task_clock.py C2 gpurun_out/task_clock_C2.json > gpurun_out/task_clock_C2.txt 2>&1 || exit 1
DYNOSAM_AMD_LIB_DIR=variants/tclk timeout -k 10 300 python tools/task_clock.py NS gpurun_out/task_clock_NS.json > gpurun_out/task_clock_NS.txt 2>&1 || exit 2
