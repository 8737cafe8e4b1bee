#!/bin/bash
# Round-4 check: the whole -m gpu suite, smoke, then C2/NS kernel-trace
# profiles and the C2 bench line. Stops at the first failing step.
set -o pipefail
o=gpurun_out/r4c
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -x > $o/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 2
bash tools/prof_run.sh $o/prof_c2 bench.py --steps 3 --no-cpu-baseline > $o/prof_c2.txt 2>&1 || exit 3
bash tools/prof_run.sh $o/prof_ns bench.py --config NS --steps 2 --no-cpu-baseline > $o/prof_ns.txt 2>&1 || exit 4
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $o/bench_c2.log 2>&1 || exit 5
