#!/bin/bash
# backward-solve part size sweep (bench lines, no profiler)
set -o pipefail
o=gpurun_out/${1:-swb}; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $o/gpu_parity.log 2>&1 || exit 1
for cfg in C2 NS; do
  for t in 2 4 8 16; do
    DYNOHIP_BACK_PART_TILES=$t timeout -k 10 200 python -u bench.py --config $cfg --steps 10 --no-cpu-baseline > $o/${cfg}_t$t.log 2>&1 || exit 2
  done
done
