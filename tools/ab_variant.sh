#!/bin/bash
# A/B of a compile-time variant (tools/build_variant.sh <dir> -D...): parity
# tests of the variant, then bench lines of the default build and the variant
# (no profiler), then a kernel-trace of the variant at C2.
# usage: tools/ab_variant.sh <variant dir> <out>
set -o pipefail
v=$1; o=gpurun_out/${2:-ab}; mkdir -p $o
[ -n "$SKIP_PARITY" ] || DYNOSAM_AMD_LIB_DIR=$v timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $o/gpu_parity_variant.log 2>&1 || exit 1
for cfg in C2 NS; do
  timeout -k 10 200 python -u bench.py --config $cfg --steps 10 --no-cpu-baseline > $o/base_$cfg.log 2>&1 || exit 2
  DYNOSAM_AMD_LIB_DIR=$v timeout -k 10 200 python -u bench.py --config $cfg --steps 10 --no-cpu-baseline > $o/var_$cfg.log 2>&1 || exit 3
done
DYNOSAM_AMD_LIB_DIR=$v bash tools/prof_run.sh $o/prof_var_C2 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $o/prof_var_C2.txt 2>&1 || exit 4
