"""Quick GPU-vs-oracle check used during development (prints diagnostics)."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
from dynosam_amd import synth
from dynosam_amd.optimizer import Solver
from oracle_binding import Oracle

names = sys.argv[1:] or ["T1", "T2", "C1"]
for name in names:
    g, v, gt = synth.generate(name)
    s = Solver(0)
    s.set_graph(g); s.set_values(v); s.set_timing(True)
    o = Oracle(g, v)
    print(f"== {name}: values {len(v)} factors {g.size()}", flush=True)
    e_gpu, e_orc = s.error(), o.error()
    print(f"error gpu {e_gpu!r} oracle {e_orc!r} rel {abs(e_gpu-e_orc)/abs(e_orc):.3e}", flush=True)
    lg, lo = s.linearize(), o.linearize()
    print(f"linearize max abs diff {np.max(np.abs(lg-lo)):.3e} (max |.| {np.max(np.abs(lo)):.3e})", flush=True)
    for it in range(3):
        sg = s.iterate(); so = o.iterate()
        dg, do = s.values_data(), o.values_data()
        rel = np.linalg.norm(dg - do) / np.linalg.norm(do)
        print(f"iter {it}: gpu it={sg.iterations} inner={sg.inner_iterations} err={sg.final_error!r} | "
              f"oracle it={so.iterations} inner={so.inner_iterations} err={so.final_error!r} | values rel {rel:.3e}", flush=True)
    s.set_values(v)
    t = time.time(); sg = s.optimize(); tg = time.time() - t
    o2 = Oracle(g, v)
    t = time.time(); so = o2.optimize(); to = time.time() - t
    rel = np.linalg.norm(s.values_data() - o2.values_data()) / np.linalg.norm(o2.values_data())
    print(f"optimize gpu it={sg.iterations} inner={sg.inner_iterations} err={sg.final_error:.6e} {tg*1e3:.1f} ms | "
          f"oracle it={so.iterations} inner={so.inner_iterations} err={so.final_error:.6e} {to*1e3:.1f} ms | rel {rel:.3e}", flush=True)
    print("stats", s.stats(), flush=True)
    s.close()
