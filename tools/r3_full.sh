#!/bin/bash
# the whole -m gpu suite, then the C2 / NS / stream bench lines and a C2 kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests > gpurun_out/full_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 10 --no-cpu-baseline > gpurun_out/full_c2.log 2>&1 || exit 2
timeout -k 10 200 python -u bench.py --config NS --steps 5 --no-cpu-baseline > gpurun_out/full_ns.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --mode stream --steps 3 --warmup 1 > gpurun_out/full_stream.log 2>&1 || exit 4
bash tools/prof_run.sh gpurun_out/full_prof_c2 bench.py --steps 3 --no-cpu-baseline > gpurun_out/full_prof_c2.txt 2>&1 || exit 5
