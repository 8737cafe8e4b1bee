#!/bin/bash
# Backward-part size sweep (DYNOHIP_BACK_PART_TILES) for k_back_poll at C2
# and NS: kernel-trace stats of a short bench per setting.
set -o pipefail
o=gpurun_out/r4bs
mkdir -p $o
for cfg in C2 NS; do
  for t in 2 4 8; do
    DYNOHIP_BACK_PART_TILES=$t bash tools/prof_run.sh $o/${cfg}_$t bench.py --config $cfg --steps 2 --no-cpu-baseline > $o/${cfg}_$t.txt 2>&1 || exit 1
  done
done
