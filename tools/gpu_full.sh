#!/bin/bash
# GPU check: all GPU tests, smoke, full-batch call breakdown, C2 bench line.
# Each step under its own limit; stops at the first failure. Outputs under gpurun_out/full/.
set -o pipefail
o=gpurun_out/full; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 2
timeout -k 10 200 python -u tools/fb_timing.py C2 3 > $o/fb.txt 2>&1 || exit 3
timeout -k 10 300 python -u bench.py > $o/bench_c2.log 2>&1 || exit 4
