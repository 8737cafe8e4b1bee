#!/bin/bash
# host planning time at C2 and NS on the box's cores (min/median over reps),
# then one rep with the per-phase breakdown
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/plan_timing.py C2 15 > gpurun_out/plan_c2_box.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/plan_timing.py NS 9 > gpurun_out/plan_ns_box.log 2>&1 || exit 2
DYNOHIP_SCHED_TIMING=1 DYNOHIP_PLAN_TIMING=1 timeout -k 10 200 python -u tools/plan_timing.py C2 4 > gpurun_out/plan_c2_box_phases.log 2>&1 || exit 3
DYNOHIP_SCHED_TIMING=1 DYNOHIP_PLAN_TIMING=1 timeout -k 10 300 python -u tools/plan_timing.py NS 4 > gpurun_out/plan_ns_box_phases.log 2>&1 || exit 4
