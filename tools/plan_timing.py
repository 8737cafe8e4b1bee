"""Host planning time of dynohip_set_graph (build_plan + tile schedule) on a
synthetic config; DYNOHIP_PLAN_TIMING=1 adds the per-phase breakdown.
usage: python tools/plan_timing.py [C2|NS|C5|...] [reps]"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynosam_amd import _abi, _native, synth  # noqa: E402

lib = _native.load("libdynohip.so")
g, v, _ = synth.generate(sys.argv[1] if len(sys.argv) > 1 else "C2")
gv = g.view()
info = _abi.ScheduleInfo()
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ts = []
for _ in range(reps):
    t = time.time()
    lib.dynohip_plan_schedule(C.byref(gv), v.keys.ctypes.data_as(C.POINTER(C.c_uint64)),
                              v.kinds.ctypes.data_as(C.POINTER(C.c_uint8)), len(v), C.byref(info), *([None] * 12))
    ts.append((time.time() - t) * 1e3)
    print("plan total ms %.1f" % ts[-1], file=sys.stderr)
print("plan total ms min %.2f median %.2f over %d" % (min(ts), sorted(ts)[len(ts) // 2], reps), file=sys.stderr)
