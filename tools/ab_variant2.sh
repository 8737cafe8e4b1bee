#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
bash tools/prof_run.sh gpurun_out/ab_base bench.py --steps 3 --no-cpu-baseline > gpurun_out/ab_base.txt 2>&1 || exit 1
DYNOSAM_AMD_LIB_DIR=variants/band_s3 bash tools/prof_run.sh gpurun_out/ab_s3 bench.py --steps 3 --no-cpu-baseline > gpurun_out/ab_s3.txt 2>&1 || exit 2
bash tools/prof_run.sh gpurun_out/ab_base_ns bench.py --config NS --steps 3 --no-cpu-baseline > gpurun_out/ab_base_ns.txt 2>&1 || exit 3
DYNOSAM_AMD_LIB_DIR=variants/band_s3 bash tools/prof_run.sh gpurun_out/ab_s3_ns bench.py --config NS --steps 3 --no-cpu-baseline > gpurun_out/ab_s3_ns.txt 2>&1 || exit 4
