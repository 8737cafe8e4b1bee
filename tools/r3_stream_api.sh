#!/bin/bash
# HIP API + kernel trace of one sliding-window stream replay (host timeline
# of a window solve), and the plan/values timing lines of one replay.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -d gpurun_out/api_stream -o run --output-format csv -- python -u bench.py --mode stream --steps 1 --warmup 0 > gpurun_out/api_stream.log 2>&1 || exit 1
DYNOHIP_PLAN_TIMING=1 timeout -k 10 200 python -u bench.py --mode stream --steps 1 --warmup 0 > gpurun_out/stream_plan_timing.log 2>&1 || exit 2
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_backend.py tests/test_c_abi.py -m gpu > gpurun_out/api_tests.log 2>&1 || exit 3
