#!/bin/bash
# Stream bench after the object-pose propagation change (construction
# included), two runs; the backend -m gpu tests.
set -o pipefail
o=gpurun_out/r4s
mkdir -p $o
timeout -k 10 300 python -u bench.py --mode stream --steps 2 --warmup 1 > $o/bench_stream_sw.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --mode stream --steps 2 --warmup 1 > $o/bench_stream_sw2.log 2>&1 || exit 2
timeout -k 10 600 python -u -m pytest tests/test_backend.py tests/test_replay.py -m gpu -q --timeout 400 --timeout-method thread -x > $o/gpu_tests_backend.log 2>&1 || exit 3
