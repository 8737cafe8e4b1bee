#!/bin/bash
# per-rank partitioned planning time at C5 (2 ranks), with the phase breakdown of one rank
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/plan_timing_part.py C5 2 3 > gpurun_out/c5_plan.log 2>&1 || exit 1
DYNOHIP_PLAN_TIMING=1 DYNOHIP_SCHED_TIMING=1 timeout -k 10 300 python -u tools/plan_timing_part.py C5 2 3 > gpurun_out/c5_plan_phases.log 2>&1 || exit 2
