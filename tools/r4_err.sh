#!/bin/bash
# k_error at 4 (compiler's choice), 6 and 8 waves per SIMD (variants/err6,
# variants/err8: spilling Between's registers); NS and C2 kernel stats; then
# the -m gpu suite and smoke() on the final build.
set -o pipefail
o=gpurun_out/r4e
mkdir -p $o
bash tools/prof_run.sh $o/prof_ns bench.py --config NS --steps 2 --no-cpu-baseline > $o/prof_ns.txt 2>&1 || exit 1
DYNOSAM_AMD_LIB_DIR=variants/err6 bash tools/prof_run.sh $o/prof_ns6 bench.py --config NS --steps 2 --no-cpu-baseline > $o/prof_ns6.txt 2>&1 || exit 2
DYNOSAM_AMD_LIB_DIR=variants/err8 bash tools/prof_run.sh $o/prof_ns8 bench.py --config NS --steps 2 --no-cpu-baseline > $o/prof_ns8.txt 2>&1 || exit 3
bash tools/prof_run.sh $o/prof_c2 bench.py --steps 3 --no-cpu-baseline > $o/prof_c2.txt 2>&1 || exit 4
DYNOSAM_AMD_LIB_DIR=variants/err8 bash tools/prof_run.sh $o/prof_c2_8 bench.py --steps 3 --no-cpu-baseline > $o/prof_c2_8.txt 2>&1 || exit 5
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -x > $o/gpu_tests.log 2>&1 || exit 6
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 7
