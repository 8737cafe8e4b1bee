#!/bin/bash
# round-3 end (part B): PMC passes + kernel stats at C2/NS, the full-batch
# call breakdown, partitioned tests, per-rank planning at C5, stream trace
set -o pipefail
mkdir -p gpurun_out/final
bash tools/pmc_passes.sh gpurun_out/final/pmc_C2 C2 --steps 3 --no-cpu-baseline || exit 1
bash tools/pmc_passes.sh gpurun_out/final/pmc_NS NS --config NS --steps 3 --no-cpu-baseline || exit 2
timeout -k 10 200 python -u tools/fb_timing.py C2 4 > gpurun_out/final/fb_timing_c2.log 2>&1 || exit 3
timeout -k 10 300 python -u tools/plan_timing_part.py C5 2 > gpurun_out/final/plan_c5_part.log 2>&1 || exit 4
timeout -k 10 560 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_partition.py -m gpu > gpurun_out/final/part_tests.log 2>&1 || exit 5
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/final/prof_stream -o run --output-format csv -- python3 -u bench.py --mode stream --steps 1 --warmup 1 > gpurun_out/final/prof_stream.log 2>&1 || exit 6
