"""Host half of the reference's full-batch unit (RGBDBackendModule.cc:217-221):
set_graph / set_values (planning + upload) / optimize / values read back, per
call on a persistent handle, for C2 and NS. Run with DYNOHIP_PLAN_TIMING=1 for
the planner's own phase marks on stderr. Usage: python tools/host_timing.py [C2 NS]"""
import sys
import time

sys.path.insert(0, ".")
from dynosam_amd import synth  # noqa: E402
from dynosam_amd.optimizer import Solver  # noqa: E402


def main(names):
    for name in names:
        g, v, _ = synth.generate(name)
        s = Solver(0)
        for rep in range(4):
            t0 = time.perf_counter()
            s.set_graph(g)
            t1 = time.perf_counter()
            s.set_values(v)
            t2 = time.perf_counter()
            r = s.optimize()
            t3 = time.perf_counter()
            s.values_data()
            t4 = time.perf_counter()
            print(f"{name} call {rep}: set_graph {1e3 * (t1 - t0):.2f} ms, set_values (plan + upload) "
                  f"{1e3 * (t2 - t1):.2f} ms, optimize {1e3 * (t3 - t2):.2f} ms ({r.iterations} it), "
                  f"values {1e3 * (t4 - t3):.2f} ms, total {1e3 * (t4 - t0):.2f} ms", flush=True)
            print(f"{name} call {rep} done", file=sys.stderr, flush=True)
        s.close()


if __name__ == "__main__":
    main(sys.argv[1:] or ["C2", "NS"])
