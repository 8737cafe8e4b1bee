#!/bin/bash
# one GPU test by -k expression: bash tools/r3_gpu_one.sh EXPR
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$1" > gpurun_out/gpu_one.log 2>&1 || exit 1
