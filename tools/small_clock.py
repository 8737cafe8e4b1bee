"""Timeline of one k_small_solve launch (the one-workgroup window solve).

Needs a libdynohip.so built with -DDYNOHIP_TASK_CLOCK (tools/build_variant.sh
<dir> -DDYNOHIP_TASK_CLOCK, then DYNOSAM_AMD_LIB_DIR=<dir>) and
DYNOHIP_SMALL_SOLVE=1. Solves one damped system of a 10-frame window-sized
graph (four tiles) and prints, in shader cycles (s_memtime) from the first
stamp: per diagonal block K, wave 0's factor start, W_K out, hand-over
received, step end, and x_K out in the backward pass; per wave, when each step
was done.

usage: python tools/small_clock.py
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from dynosam_amd import _native, synth  # noqa: E402
from dynosam_amd.optimizer import Solver  # noqa: E402


def main():
    g, v, _ = synth.generate(None, frames=10, objects=3, static_landmarks=150, dyn_slots=6)
    s = Solver(0)
    s.set_graph(g)
    s.set_values(v)
    for _ in range(3):
        ok, _ = s.solve_delta(1e-3)
        assert ok
    lib = _native.load("libdynohip.so")
    buf = np.zeros((32, 32768), dtype=np.uint64)
    lib.dynohip_debug_task_clock.argtypes = [C.c_void_p, C.c_int]
    assert lib.dynohip_debug_task_clock(buf.ctypes.data, 1) >= 0
    t = buf.astype(np.int64)
    t0 = t[28, :16].min()
    rel = lambda x: (x - t0)  # noqa: E731
    print("start per wave:", rel(t[28, :16]).tolist())
    print("end per wave:  ", rel(t[29, :16]).tolist())
    print(" K  factor_start  W_out  handover  step_end  x_out  | factor  wait_ho  tail")
    for K in range(16):
        a, b_, c, d, x = (rel(t[i, K]) for i in (20, 21, 22, 23, 24))
        print(f"{K:2d} {a:12d} {b_:7d} {c:9d} {d:9d} {x:7d}  | {b_ - a:6d} {c - b_:7d} {d - c:6d}")
    print("hand-over sent (J):", [int(rel(t[27, J])) for J in range(1, 16)])
    print("step done per wave (rows: wave 1..15, cols K):")
    for w in range(1, 16):
        print(f"w{w:2d}", " ".join(f"{int(rel(t[25, 16 * w + K])):6d}" for K in range(16)))
    print("W_K seen per wave:")
    for w in range(1, 16):
        print(f"w{w:2d}", " ".join(f"{int(rel(t[26, 16 * w + K])):6d}" for K in range(16)))
    s.close()


if __name__ == "__main__":
    main()
