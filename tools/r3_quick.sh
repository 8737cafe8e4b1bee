#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/q_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 10 --no-cpu-baseline > gpurun_out/q_c2.log 2>&1 || exit 2
bash tools/prof_run.sh gpurun_out/q_prof_c2 bench.py --steps 3 --no-cpu-baseline > gpurun_out/q_prof_c2.txt 2>&1 || exit 3
