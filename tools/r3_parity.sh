#!/bin/bash
# Round-3 parity probe: the new/extended oracle comparisons (C2 all
# iterations, solve_delta, NS/C5 conditioned, LLWorld gauge checks, C5
# partitioned vs oracle), printed (-s) into gpurun_out/r3_parity.log.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 560 python -u -m pytest -s -v --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_c_abi.py "tests/test_partition.py::test_partitioned_c5_two_ranks" > gpurun_out/r3_parity.log 2>&1
