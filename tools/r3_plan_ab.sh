#!/bin/bash
# planner pool spin A/B at C2 and NS (min/median over reps)
set -o pipefail
mkdir -p gpurun_out
for sp in 0 500 100 2000 0 500; do
  echo "spin_us=$sp" >> gpurun_out/plan_ab.log
  DYNOHIP_PLAN_SPIN_US=$sp timeout -k 10 200 python -u tools/plan_timing.py C2 15 2>&1 | tail -n 1 >> gpurun_out/plan_ab.log || exit 1
  DYNOHIP_PLAN_SPIN_US=$sp timeout -k 10 300 python -u tools/plan_timing.py NS 9 2>&1 | tail -n 1 >> gpurun_out/plan_ab.log || exit 2
done
