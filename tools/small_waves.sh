#!/bin/bash
# The one-workgroup window solve with 16 waves (variants/small16) against the
# default 8: its test, then the window stream's kernel trace with it on.
set -o pipefail
o=gpurun_out/smallw
mkdir -p $o
DYNOSAM_AMD_LIB_DIR=variants/small16 timeout -k 10 240 python -u -m pytest tests/test_gpu_parity.py -k small_solve -v -s --timeout 120 --timeout-method thread -x > $o/test16.log 2>&1 || exit 1
DYNOHIP_SMALL_SOLVE=1 DYNOSAM_AMD_LIB_DIR=variants/small16 bash tools/prof_run.sh $o/prof16 bench.py --mode stream --steps 1 --warmup 0 > $o/prof16.txt 2>&1 || exit 2
DYNOHIP_SMALL_SOLVE=1 bash tools/prof_run.sh $o/prof8 bench.py --mode stream --steps 1 --warmup 0 > $o/prof8.txt 2>&1 || exit 3
