#!/bin/bash
# full-batch call at C2 under planner pool settings (workers, spin), interleaved
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/fb_sweep.txt
for round in 1 2; do
  for cfg in "16 500" "12 500" "8 500" "16 100" "12 2000"; do
    set -- $cfg
    DYNOHIP_PLAN_WORKERS=$1 DYNOHIP_PLAN_SPIN_US=$2 timeout -k 10 200 python -u tools/fb_timing.py C2 8 > gpurun_out/fbs.log 2>&1 || exit 1
    python tools/fb_summary.py gpurun_out/fbs.log "w=$1 spin=$2" >> gpurun_out/fb_sweep.txt
  done
done
