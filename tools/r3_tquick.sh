#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "queue_order or cost_change" > gpurun_out/t_tests.log 2>&1 || exit 1
