#!/bin/bash
# A/B of the linearised cost change: from the solve (default) vs k_linerr
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/ab_tests.log 2>&1 || exit 1
DYNOHIP_LINERR_DIRECT=1 bash tools/prof_run.sh gpurun_out/ab_direct bench.py --steps 3 --no-cpu-baseline > gpurun_out/ab_direct.txt 2>&1 || exit 2
bash tools/prof_run.sh gpurun_out/ab_fused bench.py --steps 3 --no-cpu-baseline > gpurun_out/ab_fused.txt 2>&1 || exit 3
timeout -k 10 200 python -u bench.py --steps 10 --no-cpu-baseline > gpurun_out/ab_c2.log 2>&1 || exit 4
