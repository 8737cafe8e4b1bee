#!/bin/bash
# Correctness half of tools/gpu_round.sh: the -m gpu suite and smoke().
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py > gpurun_out/bench_c2.log 2>&1 || exit 3
