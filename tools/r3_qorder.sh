#!/bin/bash
# dataflow queue order: C2/NS bench (list-scheduled vs level order), task clocks
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
timeout -k 10 200 python -u bench.py --steps 10 --no-cpu-baseline > gpurun_out/q_c2_$rep.log 2>&1 || exit 2
timeout -k 10 200 python -u bench.py --config NS --steps 5 --no-cpu-baseline > gpurun_out/q_ns_$rep.log 2>&1 || exit 3
DYNOHIP_QUEUE_ORDER=level timeout -k 10 200 python -u bench.py --steps 10 --no-cpu-baseline > gpurun_out/q_c2_level_$rep.log 2>&1 || exit 4
DYNOHIP_QUEUE_ORDER=level timeout -k 10 200 python -u bench.py --config NS --steps 5 --no-cpu-baseline > gpurun_out/q_ns_level_$rep.log 2>&1 || exit 5
done
DYNOSAM_AMD_LIB_DIR=variants/tclk timeout -k 10 200 python tools/task_clock.py C2 gpurun_out/task_clock_C2.json > gpurun_out/task_clock_C2.txt 2>&1 || exit 6
DYNOSAM_AMD_LIB_DIR=variants/tclk timeout -k 10 300 python tools/task_clock.py NS gpurun_out/task_clock_NS.json > gpurun_out/task_clock_NS.txt 2>&1 || exit 7
