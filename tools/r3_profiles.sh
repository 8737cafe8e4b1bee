#!/bin/bash
# round-3 profiles: kernel-trace stats + PMC passes (FETCH/WRITE/FP64 MFMA) at C2 and NS
set -o pipefail
mkdir -p gpurun_out
bash tools/pmc_passes.sh gpurun_out/pmc_C2 C2 --steps 3 --no-cpu-baseline || exit 1
bash tools/pmc_passes.sh gpurun_out/pmc_NS NS --config NS --steps 3 --no-cpu-baseline || exit 2
