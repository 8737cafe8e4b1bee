#!/bin/bash
# usage: tools/build_variant.sh <outdir> [-DKNOB=value ...]
# Builds libdynohip.so with compile-time kernel knobs into <outdir> (plus a
# copy of libdynosynth.so) for A/B runs: DYNOSAM_AMD_LIB_DIR=<outdir> python bench.py
set -e
root=$(cd "$(dirname "$0")/.." && pwd)
out=$(realpath -m "$1"); shift
mkdir -p "$out"
cd "$root/dynosam_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall "$@" -o "$out/libdynohip.so" \
  kernels.hip tilechol.hip solver.cpp plan.cpp tiles.cpp partition.cpp keys.cpp driver.cpp backend.cpp replay.cpp refine.hip
cp "$root/dynosam_amd/lib/libdynosynth.so" "$out/"
