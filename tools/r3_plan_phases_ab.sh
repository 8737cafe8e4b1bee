#!/bin/bash
# per-phase planning times of two planner builds on one box
set -o pipefail
mkdir -p gpurun_out
for v in base cur base cur; do
  DYNOSAM_AMD_LIB_DIR=variants/plan_$v DYNOHIP_SCHED_TIMING=1 DYNOHIP_PLAN_TIMING=1 timeout -k 10 200 python -u tools/plan_timing.py C2 8 >> gpurun_out/phases_c2_$v.log 2>&1 || exit 1
  DYNOSAM_AMD_LIB_DIR=variants/plan_$v DYNOHIP_SCHED_TIMING=1 DYNOHIP_PLAN_TIMING=1 timeout -k 10 300 python -u tools/plan_timing.py NS 5 >> gpurun_out/phases_ns_$v.log 2>&1 || exit 2
done
