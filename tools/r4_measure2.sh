#!/bin/bash
# Round-4 measurement, second part: PMC passes (FETCH/WRITE/FP64 MFMA) of
# C2 and NS, the NS bench line, and the host half of one full-batch call
# (planning phase marks on stderr). Each step under its own time limit;
# stops at the first failing step.
set -o pipefail
o=gpurun_out/r4m
mkdir -p $o
bash tools/pmc_passes.sh $o/pmc_c2 C2 --steps 3 --no-cpu-baseline || exit 1
bash tools/pmc_passes.sh $o/pmc_ns NS --config NS --steps 2 --no-cpu-baseline || exit 2
timeout -k 10 300 python -u bench.py --config NS --no-cpu-baseline > $o/bench_ns.log 2>&1 || exit 3
DYNOHIP_PLAN_TIMING=1 timeout -k 10 300 python -u tools/host_timing.py C2 NS > $o/host_timing.log 2> $o/host_timing_phases.log || exit 4
timeout -k 10 300 python -u bench.py --mode stream --steps 2 --warmup 1 > $o/bench_stream_sw.log 2>&1 || exit 5
bash tools/prof_run.sh $o/prof_stream bench.py --mode stream --steps 1 --warmup 0 > $o/prof_stream.txt 2>&1 || exit 6
bash tools/prof_run.sh $o/prof_c2 bench.py --steps 3 --no-cpu-baseline > $o/prof_c2.txt 2>&1 || exit 7
