"""C2 late iterations: each solve's backward error against its OWN
linearisation, and the GPU-vs-oracle linearisation difference (test
infrastructure)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from r3_diag2 import sparse_system, bwd, rel  # noqa: E402  (runs nothing at import? guarded below)
from dynosam_amd import synth  # noqa: E402
from dynosam_amd.optimizer import Solver  # noqa: E402
from oracle_binding import Oracle  # noqa: E402

g, v, _ = synth.generate("C2")
s = Solver(0)
s.set_graph(g)
s.set_values(v)
p = Solver(0)
p.set_graph(g)
p.set_values(v)
o = Oracle(g, v, threads=16)
s.reset()
o.reset()
for it in range(15):
    start = s.values_data()
    o.set_values_data(start)
    n0 = len(s.trace())
    sg, so = s.iterate(), o.iterate()
    lam = s.trace()[-1]["lam"]
    if it in (0, 4, 9, 13):
        p.set_values(v.with_data(start))
        lg = p.linearize()
        okg, dg = p.solve_delta(lam)
        chk = Oracle(g, v, threads=16)
        chk.set_values_data(start)
        lo = chk.linearize()
        oko, do = chk.solve_damped(lam)
        Ag, bg = sparse_system(g, v, lg)
        Ao, bo = sparse_system(g, v, lo)
        d = np.abs(lg - lo)
        crel = d / np.maximum(np.abs(lo), 1e-300)
        nz = np.abs(lo) > 0
        print(it, "lam", lam, "values rel", rel(s.values_data(), o.values_data()), "step rel", rel(dg, do), flush=True)
        print("   bwd own: gpu", bwd(Ag, bg, lam, dg), "oracle", bwd(Ao, bo, lam, do),
              "| cross: gpu step vs oracle system", bwd(Ao, bo, lam, dg), "oracle step vs gpu system", bwd(Ag, bg, lam, do))
        print("   lin diff: max abs", d.max(), "componentwise rel p50/p99/max", np.percentile(crel[nz], 50),
              np.percentile(crel[nz], 99), crel[nz].max(), flush=True)
        # the oracle solving the GPU's own linearisation? (not exposed) -> solve both systems exactly in scipy
