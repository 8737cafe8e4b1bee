#!/bin/bash
# Round-4 check: the small-system solve first (new kernel), the whole -m gpu
# suite, smoke, then the stream line and C2/NS/stream kernel-trace profiles
# and the C2 bench line. Each step under its own time limit; stops at the
# first failing step.
set -o pipefail
o=gpurun_out/r4c
mkdir -p $o
timeout -k 10 240 python -u -m pytest tests/test_gpu_parity.py -k small_solve -v --timeout 120 --timeout-method thread -x > $o/small.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -x > $o/gpu_tests.log 2>&1 || exit 2
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --mode stream --steps 2 --warmup 1 > $o/bench_stream_sw.log 2>&1 || exit 4
bash tools/prof_run.sh $o/prof_stream bench.py --mode stream --steps 1 --warmup 0 > $o/prof_stream.txt 2>&1 || exit 5
bash tools/prof_run.sh $o/prof_c2 bench.py --steps 3 --no-cpu-baseline > $o/prof_c2.txt 2>&1 || exit 6
bash tools/prof_run.sh $o/prof_ns bench.py --config NS --steps 2 --no-cpu-baseline > $o/prof_ns.txt 2>&1 || exit 7
timeout -k 10 300 python -u bench.py > $o/bench_c2.log 2>&1 || exit 8
