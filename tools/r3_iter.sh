#!/bin/bash
# one build -> measure iteration: parity subset, C2/NS bench lines, kernel trace at C2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "execution_paths or parity_conditioned or free_running or no_read or bit_repro or solve_delta" > gpurun_out/iter_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 10 --no-cpu-baseline > gpurun_out/iter_c2.log 2>&1 || exit 2
timeout -k 10 200 python -u bench.py --config NS --steps 5 --no-cpu-baseline > gpurun_out/iter_ns.log 2>&1 || exit 3
bash tools/prof_run.sh gpurun_out/iter_prof_c2 bench.py --steps 3 --no-cpu-baseline > gpurun_out/iter_prof_c2.txt 2>&1 || exit 4
