"""Per-workgroup phases of one k_lone_schur launch.

Needs a libdynohip.so built with -DDYNOHIP_LONE_CLOCK (tools/build_variant.sh
<dir> -DDYNOHIP_LONE_CLOCK, then DYNOSAM_AMD_LIB_DIR=<dir>). Runs one LM
optimisation of a synthetic config and prints, over the workgroups of the last
launch, the launch span and the distribution of each phase (s_memrealtime,
100 MHz): index block staged, point data staged, Z formed, sums done.

usage: python tools/lone_clock.py [C2|NS]
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from dynosam_amd import _native, synth  # noqa: E402
from dynosam_amd.optimizer import LevenbergMarquardtOptimizer  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
    graph, values, _ = synth.generate(cfg)
    opt = LevenbergMarquardtOptimizer(graph, values, device=0)
    opt.optimize()
    lib = _native.load("libdynohip.so")
    buf = np.zeros((8, 8192), dtype=np.uint64)
    lib.dynohip_debug_lone_clock.argtypes = [C.c_void_p]
    assert lib.dynohip_debug_lone_clock(buf.ctypes.data) == 0
    n = int(np.count_nonzero(buf[0]))
    t = buf[:5, :n].astype(np.int64)
    t = (t - t[0].min()) / 100.0
    print(f"{cfg}: {n} workgroups, launch span {t[4].max():.1f} us")
    names = ["index block", "point data", "Z", "sums + stores"]
    for i, nm in enumerate(names):
        d = t[i + 1] - t[i]
        print(f"  {nm:14s} median {np.median(d):7.2f} p90 {np.percentile(d, 90):7.2f} max {d.max():7.2f} us")
    x = (buf[5:8, :n].astype(np.int64) - buf[0, :n].astype(np.int64).min()) / 100.0
    for nm, d in (("  MFMA tiles (wave 0)", x[0] - t[3]), ("  gradient (wave 2)", x[1] - t[3]),
                  ("  barrier passed", x[2] - t[3]), ("  stores (wave 0)", t[4] - x[2])):
        print(f"  {nm:20s} median {np.median(d):7.2f} p90 {np.percentile(d, 90):7.2f} max {d.max():7.2f} us")
    tot = t[4] - t[0]
    print(f"  {'total':14s} median {np.median(tot):7.2f} p90 {np.percentile(tot, 90):7.2f} max {tot.max():7.2f} us")
    st = np.sort(t[0])
    print("  start times (percentiles 0/25/50/75/100):", np.percentile(st, [0, 25, 50, 75, 100]).round(1))


if __name__ == "__main__":
    main()
