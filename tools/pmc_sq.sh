#!/bin/bash
# usage: tools/pmc_sq.sh <outdir> <python args...>  -- one SQ stall-profile pass (kernel trace + SQ counters only)
out=$1; shift
mkdir -p $out && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD --kernel-trace -d $out -o sq --output-format csv -- python3 "$@" > $out/sq.stdout.log 2>&1
