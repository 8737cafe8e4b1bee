#!/bin/bash
# Host sanitizers over the CPU test suite: libdynohip.so rebuilt with
# -fsanitize=address (default) or, with SAN=undefined, -fsanitize=undefined
# (no recovery), on the host side only (-Xarch_host; the device code is
# unchanged), the runtime preloaded into the test process, every
# `-m "not gpu"` test run against that build (planner, module construction
# and its deferred-window threads in graphs-only mode, partitioning, replay
# reader, keys).
# usage: [SAN=undefined] tools/asan_cpu.sh [outdir]   (no GPU needed)
set -e
root=$(cd "$(dirname "$0")/.." && pwd)
san=${SAN:-address}
out=$(realpath -m "${1:-$root/build_$san}")
mkdir -p "$out"
cd "$root/dynosam_amd/csrc"
extra=()
[ "$san" = undefined ] && extra=(-Xarch_host -fno-sanitize-recover=undefined)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -shared \
  -Xarch_host -fsanitize=$san "${extra[@]}" -Xarch_host -fno-omit-frame-pointer -o "$out/libdynohip.so" \
  kernels.hip tilechol.hip solver.cpp plan.cpp tiles.cpp partition.cpp keys.cpp driver.cpp backend.cpp replay.cpp refine.hip
cp "$root/dynosam_amd/lib/libdynosynth.so" "$out/"
lib=asan
[ "$san" = undefined ] && lib=ubsan_standalone
rt=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.$lib-x86_64.so | head -1)
cd "$root"
LD_PRELOAD="$rt" ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  DYNOSAM_AMD_LIB_DIR="$out" python -m pytest tests -m "not gpu" -x -q -p no:cacheprovider
