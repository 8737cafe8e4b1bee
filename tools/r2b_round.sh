#!/bin/bash
# GPU round: full -m gpu suite, smoke, C2 bench line, kernel-trace + PMC
# passes at C2 and NS, NS bench line. Each step under its own limit; stops at
# the first failure. Outputs under gpurun_out/$1.
set -o pipefail
o=gpurun_out/${1:-r2b}; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py > $o/bench_c2.log 2>&1 || exit 3
bash tools/pmc_passes.sh $o/prof_C2 C2 --steps 3 --warmup 1 --no-cpu-baseline || exit 4
bash tools/pmc_passes.sh $o/prof_NS NS --config NS --steps 3 --warmup 1 --no-cpu-baseline || exit 5
timeout -k 10 300 python -u bench.py --config NS --no-cpu-baseline > $o/bench_ns.log 2>&1 || exit 6
