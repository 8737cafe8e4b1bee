#!/bin/bash
# usage: tools/pmc_passes.sh <outdir> <config> <bench args...>
# One kernel-trace --stats run and three PMC passes (each its own rocprofv3
# run, kernel trace only) of the same bench command, then the per-kernel
# summary (tools/pmc_summary.py). Stops at the first failing step.
out=$1; cfg=$2; shift 2
mkdir -p $out && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 bench.py "$@" > $out/trace.log 2>&1 || exit 11
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $out/fetch -o p --output-format csv -- python3 bench.py "$@" > $out/fetch.log 2>&1 || exit 12
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $out/write -o p --output-format csv -- python3 bench.py "$@" > $out/write.log 2>&1 || exit 13
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 GRBM_GUI_ACTIVE --kernel-trace -d $out/mfma -o p --output-format csv -- python3 bench.py "$@" > $out/mfma.log 2>&1 || exit 14
python3 tools/pmc_summary.py $out $cfg $out/pmc_$cfg.json > $out/summary.txt 2>&1 || exit 15
