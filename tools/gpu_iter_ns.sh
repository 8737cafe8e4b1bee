#!/bin/bash
# quick factorisation iteration: parity tests, task clock (C2, NS), C2 and NS bench lines
set -o pipefail
o=gpurun_out/t1; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_partition.py -m gpu -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1; echo tests_rc=$? >> $o/tests.log
DYNOSAM_AMD_LIB_DIR=variants/tclk timeout -k 10 150 python -u tools/task_clock.py C2 $o/c2.json > $o/c2.txt 2>&1 || exit 2
DYNOSAM_AMD_LIB_DIR=variants/tclk timeout -k 10 200 python -u tools/task_clock.py NS $o/ns.json > $o/ns.txt 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $o/bench.log 2>&1 || exit 4
timeout -k 10 300 python -u bench.py --config NS --no-cpu-baseline > $o/bench_ns.log 2>&1 || exit 5
