#!/bin/bash
# round-3 end (part A): whole -m gpu suite, smoke, the bench lines
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 700 python -u -m pytest -m gpu -q --timeout 200 --timeout-method thread tests > gpurun_out/final/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || exit 2
timeout -k 10 600 python -u bench.py > gpurun_out/final/bench_c2.log 2>&1 || exit 3
timeout -k 10 200 python -u bench.py --config NS --steps 5 --no-cpu-baseline > gpurun_out/final/bench_ns.log 2>&1 || exit 4
timeout -k 10 300 python -u bench.py --mode stream --steps 3 --warmup 1 > gpurun_out/final/bench_stream_sw.log 2>&1 || exit 5
timeout -k 10 300 python -u bench.py --mode stream --full-batch --steps 3 --warmup 1 > gpurun_out/final/bench_stream_fb.log 2>&1 || exit 6
timeout -k 10 300 python -u bench.py --mode refine > gpurun_out/final/bench_refine.log 2>&1 || exit 7
