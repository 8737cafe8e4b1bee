#!/bin/bash
# usage: tools/pmc_pass.sh <outdir> <counter> <python args...>
# One rocprofv3 PMC pass (kernel trace + one TCC counter; no sys/runtime
# trace domains), as the MI355X guide prescribes: FETCH_SIZE and WRITE_SIZE
# do not fit one pass on gfx950.
out=$1; ctr=$2; shift 2
mkdir -p $out && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --pmc $ctr --kernel-trace -d $out -o $ctr --output-format csv -- python3 "$@" > $out/$ctr.stdout.log 2>&1
