#!/bin/bash
# GPU check: parity tests, smoke, C2 bench line, C2 kernel-trace stats.
# Each step under its own limit; stops at the first failure. Outputs under
# gpurun_out/$1 (default chk).
set -o pipefail
o=gpurun_out/${1:-chk}; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py > $o/bench_c2.log 2>&1 || exit 3
bash tools/prof_run.sh $o/prof_C2 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $o/prof_C2.txt 2>&1 || exit 4
bash tools/prof_run.sh $o/prof_NS bench.py --config NS --steps 3 --warmup 1 --no-cpu-baseline > $o/prof_NS.txt 2>&1 || exit 5
