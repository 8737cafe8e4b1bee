#!/bin/bash
# Queue-order cost model sweep (DYNOHIP_QCOST="panel,update,pair,handoff"):
# the factorisation's per-launch time in the NS and C2 bench lines.
set -o pipefail
o=gpurun_out/qcost
mkdir -p $o
for cfg in NS C2; do
  for qc in "16,5.5,1.7,2.5" "17,6.2,1.7,3.5" "17,8,2,5" "17,11,2,7"; do
    DYNOHIP_QCOST=$qc timeout -k 10 200 python -u bench.py --config $cfg --steps 2 --no-cpu-baseline > $o/bench_${cfg}_${qc}.log 2>&1 || exit 1
    python - $o/bench_${cfg}_${qc}.log $cfg $qc <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith('{'):
        d = json.loads(line)
        print(sys.argv[2], sys.argv[3], "factor ms", round(d["roofline"]["ms_per_launch"], 4), "LM it/s", round(d["value"], 1))
PY
  done
done
