#!/bin/bash
# Round-4 measurement: C2 and NS bench lines, kernel-trace profiles, PMC
# passes (FETCH/WRITE/FP64 MFMA) of C2 and NS, the stream lines. Each step
# under its own time limit; stops at the first failing step.
set -o pipefail
o=gpurun_out/r4
mkdir -p $o
timeout -k 10 300 python -u bench.py > $o/bench_c2.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config NS --no-cpu-baseline > $o/bench_ns.log 2>&1 || exit 2
bash tools/prof_run.sh $o/prof_c2 bench.py --steps 3 --no-cpu-baseline > $o/prof_c2.txt 2>&1 || exit 3
bash tools/prof_run.sh $o/prof_ns bench.py --config NS --steps 2 --no-cpu-baseline > $o/prof_ns.txt 2>&1 || exit 4
bash tools/pmc_passes.sh $o/pmc_c2 C2 --steps 3 --no-cpu-baseline || exit 5
bash tools/pmc_passes.sh $o/pmc_ns NS --config NS --steps 2 --no-cpu-baseline || exit 6
timeout -k 10 300 python -u bench.py --mode stream --steps 2 --warmup 1 > $o/bench_stream_sw.log 2>&1 || exit 7
bash tools/prof_run.sh $o/prof_stream bench.py --mode stream --steps 1 --warmup 0 > $o/prof_stream.txt 2>&1 || exit 8
