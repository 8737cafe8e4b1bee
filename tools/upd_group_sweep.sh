#!/bin/bash
# Update-task grouping sweep (DYNOHIP_UPD_GROUP = levels of contributions
# per update task): the factorisation's per-launch time in the bench lines.
set -o pipefail
o=gpurun_out/updgroup
mkdir -p $o
for cfg in NS C2; do
  for g in 1 2 3 4 6 8; do
    DYNOHIP_UPD_GROUP=$g timeout -k 10 200 python -u bench.py --config $cfg --steps 2 --no-cpu-baseline > $o/bench_${cfg}_$g.log 2>&1 || exit 1
    python - $o/bench_${cfg}_$g.log $cfg $g <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith('{'):
        d = json.loads(line)
        print(sys.argv[2], "group", sys.argv[3], "factor ms", round(d["roofline"]["ms_per_launch"], 4), "LM it/s", round(d["value"], 1))
PY
  done
done
