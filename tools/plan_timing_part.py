"""Host planning time of one rank's partitioned plan (build_partitioned_plan,
as dynohip_set_values runs it on a handle with nranks > 1) for a synthetic
config: one build per measurement (dynohip_plan_export's size query; the
optimizer's plan_export builds twice, size then data).
usage: python tools/plan_timing_part.py [C5] [nranks] [reps]"""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynosam_amd import _native, synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C5"
nr = int(sys.argv[2]) if len(sys.argv) > 2 else 2
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
lib = _native.load("libdynohip.so")
t = time.time()
g, v, _ = synth.generate(cfg)
print(f"{cfg}: generate {time.time() - t:.2f} s", flush=True)
gv = g.view()
keys = np.ascontiguousarray(v.keys, dtype=np.uint64)
kinds = np.ascontiguousarray(v.kinds, dtype=np.uint8)


def build(nranks, rank):
    n = C.c_size_t()
    t = time.time()
    rc = lib.dynohip_plan_export(C.byref(gv), keys.ctypes.data_as(C.POINTER(C.c_uint64)),
                                 kinds.ctypes.data_as(C.POINTER(C.c_uint8)), keys.shape[0], nranks, rank,
                                 b"info", None, 0, C.byref(n))
    assert rc == 0, rc
    return time.time() - t


for rep in range(reps):
    for rank in range(nr):
        print(f"{cfg} nranks={nr} rank={rank}: plan {build(nr, rank):.3f} s", flush=True)
print(f"{cfg} single handle: plan {build(1, 0):.3f} s", flush=True)
