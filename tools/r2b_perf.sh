#!/bin/bash
# Quick GPU perf iteration: core parity tests, C2 and NS kernel-trace stats.
# Outputs under gpurun_out/$1.
set -o pipefail
o=gpurun_out/${1:-perf}; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $o/gpu_parity.log 2>&1 || exit 1
bash tools/prof_run.sh $o/prof_C2 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $o/prof_C2.txt 2>&1 || exit 4
bash tools/prof_run.sh $o/prof_NS bench.py --config NS --steps 3 --warmup 1 --no-cpu-baseline > $o/prof_NS.txt 2>&1 || exit 5
