#!/bin/bash
# planner A/B on one box: variants/plan_{base,cur} (min/median over reps),
# cur also with the pool's spin off; then per-phase logs of cur
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/plan_ab.log
for round in 1 2; do
  for v in base prev cur; do
    d=variants/plan_$v; sp=500
    
    echo "variant=$v" >> gpurun_out/plan_ab.log
    DYNOSAM_AMD_LIB_DIR=$d DYNOHIP_PLAN_SPIN_US=$sp timeout -k 10 200 python -u tools/plan_timing.py C2 15 2>&1 | tail -n 1 >> gpurun_out/plan_ab.log || exit 1
    DYNOSAM_AMD_LIB_DIR=$d DYNOHIP_PLAN_SPIN_US=$sp timeout -k 10 300 python -u tools/plan_timing.py NS 7 2>&1 | tail -n 1 >> gpurun_out/plan_ab.log || exit 2
  done
done
rm -f gpurun_out/phases_*
for v in base cur; do
  DYNOSAM_AMD_LIB_DIR=variants/plan_$v DYNOHIP_SCHED_TIMING=1 DYNOHIP_PLAN_TIMING=1 timeout -k 10 200 python -u tools/plan_timing.py C2 8 >> gpurun_out/phases_c2_$v.log 2>&1 || exit 3
  DYNOSAM_AMD_LIB_DIR=variants/plan_$v DYNOHIP_SCHED_TIMING=1 DYNOHIP_PLAN_TIMING=1 timeout -k 10 300 python -u tools/plan_timing.py NS 5 >> gpurun_out/phases_ns_$v.log 2>&1 || exit 4
done
