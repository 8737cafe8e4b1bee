#!/bin/bash
# Round-4 closing check of the final tree: the -m gpu suite and smoke().
set -o pipefail
o=gpurun_out/r4close
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -x > $o/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 2
