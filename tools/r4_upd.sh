#!/bin/bash
# Update-task operand prefetch: parity tests touching the factorisation,
# then the NS and C2 factorisation times.
set -o pipefail
o=gpurun_out/r4u
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -x -k "execution_paths or queue_order or conditioned_vs_oracle_at_scale or per_iteration_parity" > $o/parity.log 2>&1 || exit 1
for cfg in NS C2; do
  timeout -k 10 200 python -u bench.py --config $cfg --steps 3 --no-cpu-baseline > $o/bench_$cfg.log 2>&1 || exit 2
  python - $o/bench_$cfg.log $cfg <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith('{'):
        d = json.loads(line)
        print(sys.argv[2], "factor ms", round(d["roofline"]["ms_per_launch"], 4), "LM it/s", round(d["value"], 1))
PY
done
