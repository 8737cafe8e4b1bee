"""Factorisation time per nested-dissection leaf size (GPU): for each leaf,
plan, run LM iterations and report the per-solve factorisation and backward
times and the levels. usage: python tools/leaf_sweep.py [C2|NS] leaf..."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynosam_amd import synth  # noqa: E402
from dynosam_amd.optimizer import Solver, set_tile_ordering  # noqa: E402

cfg = sys.argv[1]
graph, values, _ = synth.generate(cfg)
for leaf in [int(x) for x in sys.argv[2:]]:
    set_tile_ordering(leaf)
    s = Solver(0)
    s.set_graph(graph)
    s.set_values(values)
    s.snapshot()
    best = None
    for _ in range(4):
        s.restore()
        t0 = time.perf_counter()
        r = s.optimize()
        dt = (time.perf_counter() - t0) * 1e3 / max(r.inner_iterations, 1)
        best = dt if best is None else min(best, dt)
    s.set_timing(True)
    s.restore()
    r = s.optimize()
    st = s.stats()
    n = max(r.inner_iterations, 1)
    print(f"{cfg} leaf={leaf} nd_leaf={st['nd_leaf']} levels={st['chol_levels']} tiles={st['tiles_stored']} "
          f"iters={r.iterations} ms_per_inner={best:.4f} factor_ms={st['ms_cholesky'] / n:.4f} "
          f"backward_ms={st['ms_solve'] / n:.4f}", flush=True)
    s.close()
set_tile_ordering(-1)
