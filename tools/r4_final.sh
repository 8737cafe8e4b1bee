#!/bin/bash
# Round-4 final measurements: PMC passes and kernel traces of C2 and NS, the
# C2 (with the CPU baseline and NS leg), NS and stream bench lines, the
# stream kernel trace. Each step under its own time limit.
set -o pipefail
o=gpurun_out/r4f
mkdir -p $o
bash tools/pmc_passes.sh $o/pmc_c2 C2 --steps 3 --no-cpu-baseline || exit 1
bash tools/pmc_passes.sh $o/pmc_ns NS --config NS --steps 2 --no-cpu-baseline || exit 2
timeout -k 10 300 python -u bench.py --config NS --no-cpu-baseline > $o/bench_ns.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --mode stream --steps 2 --warmup 1 > $o/bench_stream_sw.log 2>&1 || exit 4
bash tools/prof_run.sh $o/prof_stream bench.py --mode stream --steps 1 --warmup 0 > $o/prof_stream.txt 2>&1 || exit 5
timeout -k 10 300 python -u bench.py > $o/bench_c2.log 2>&1 || exit 6
