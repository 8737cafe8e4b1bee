#!/bin/bash
# One GPU verification round: parity tests, smoke, C2/NS bench lines and a
# C2 kernel-trace profile, each step under its own time limit; stops at the
# first failure. Outputs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py > gpurun_out/bench_c2.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --config NS --no-cpu-baseline > gpurun_out/bench_ns.log 2>&1 || exit 4
bash tools/prof_run.sh gpurun_out/prof_c2 bench.py --steps 3 --no-cpu-baseline > gpurun_out/prof_c2.txt 2>&1 || exit 5
timeout -k 10 300 python -u bench.py --mode stream --steps 2 --warmup 1 > gpurun_out/bench_stream_sw.log 2>&1 || exit 6
timeout -k 10 300 python -u bench.py --mode stream --full-batch --steps 2 --warmup 1 > gpurun_out/bench_stream_fb.log 2>&1 || exit 7
timeout -k 10 300 python -u bench.py --mode refine --steps 3 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_refine.log 2>&1 || exit 8
bash tools/prof_run.sh gpurun_out/prof_refine bench.py --mode refine --steps 2 --no-cpu-baseline > gpurun_out/prof_refine.txt 2>&1 || exit 9
