#!/bin/bash
# rocprofv3 kernel-trace stats + PMC passes (tools/pmc_passes.sh) for C2 and
# NS with the current build; summaries under gpurun_out/prof/. Stops at the
# first failing step.
set -o pipefail
o=gpurun_out/prof; mkdir -p $o
bash tools/pmc_passes.sh $o/C2 C2 --steps 3 --warmup 1 --no-cpu-baseline || exit 4
bash tools/pmc_passes.sh $o/NS NS --config NS --steps 3 --warmup 1 --no-cpu-baseline || exit 5
