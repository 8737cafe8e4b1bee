"""Host planning time of one rank's partitioned plan (build_partitioned_plan,
as dynohip_set_values runs it on a handle with nranks > 1) for a synthetic
config. usage: python tools/plan_timing_part.py [C5] [nranks]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynosam_amd import synth  # noqa: E402
from dynosam_amd.optimizer import plan_export  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C5"
nr = int(sys.argv[2]) if len(sys.argv) > 2 else 2
t = time.time()
g, v, _ = synth.generate(cfg)
print(f"{cfg}: generate {time.time() - t:.2f} s", flush=True)
for rep in range(3):
    for rank in range(nr):
        t = time.time()
        plan_export(g, v, "info", nranks=nr, rank=rank)
        print(f"{cfg} nranks={nr} rank={rank}: plan {time.time() - t:.3f} s", flush=True)
t = time.time()
plan_export(g, v, "info")
print(f"{cfg} single handle: plan {time.time() - t:.3f} s", flush=True)
