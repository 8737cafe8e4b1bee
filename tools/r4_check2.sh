#!/bin/bash
# Round-4 check after the update grouping: the -m gpu suite, then the NS and
# C2 bench lines and the NS kernel-trace profile.
set -o pipefail
o=gpurun_out/r4c2
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -x > $o/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config NS --no-cpu-baseline > $o/bench_ns.log 2>&1 || exit 2
bash tools/prof_run.sh $o/prof_ns bench.py --config NS --steps 2 --no-cpu-baseline > $o/prof_ns.txt 2>&1 || exit 3
timeout -k 10 300 python -u bench.py > $o/bench_c2.log 2>&1 || exit 4
