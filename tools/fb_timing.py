"""Breakdown of one full-batch call as the reference times it
(RGBDBackendModule.cc:217-221): handle creation, set_graph, set_values
(host planning + upload), optimize, values read back, destroy.
usage: python tools/fb_timing.py [C2|NS] [repeats]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynosam_amd import synth  # noqa: E402
from dynosam_amd.optimizer import Solver  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
graph, values, _ = synth.generate(cfg)
print("fresh handle per call:")
for rep in range(reps):
    t = [time.perf_counter()]
    s = Solver(0); t.append(time.perf_counter())
    s.set_graph(graph); t.append(time.perf_counter())
    s.set_values(values); t.append(time.perf_counter())
    s.optimize(); t.append(time.perf_counter())
    s.values_data(); t.append(time.perf_counter())
    s.close(); t.append(time.perf_counter())
    names = ["create", "set_graph", "set_values", "optimize", "get_values", "destroy"]
    print(cfg, " ".join(f"{n}={1e3 * (t[i + 1] - t[i]):.2f}" for i, n in enumerate(names)),
          f"total={1e3 * (t[-1] - t[0]):.2f} ms", flush=True)
print("persistent handle (buffers reused across calls):")
s = Solver(0)
for rep in range(reps):
    t = [time.perf_counter()]
    s.set_graph(graph); t.append(time.perf_counter())
    s.set_values(values); t.append(time.perf_counter())
    s.optimize(); t.append(time.perf_counter())
    s.values_data(); t.append(time.perf_counter())
    names = ["set_graph", "set_values", "optimize", "get_values"]
    print(cfg, " ".join(f"{n}={1e3 * (t[i + 1] - t[i]):.2f}" for i, n in enumerate(names)),
          f"total={1e3 * (t[-1] - t[0]):.2f} ms", flush=True)
s.close()
