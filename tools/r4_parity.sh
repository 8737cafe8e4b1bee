#!/bin/bash
# Round-4 parity record (verbose, printed comparisons) and the C2 bench line
# with the current defaults. Each step under its own time limit.
set -o pipefail
o=gpurun_out/r4p
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -s --timeout 300 --timeout-method thread > $o/gpu_parity.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $o/bench_c2.log 2>&1 || exit 2
