"""Round-3 diagnostics (GPU box): LLWorld divergences and the C2 late-iteration
conditioning. Test infrastructure (imports the oracle)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from dynosam_amd import _abi, synth  # noqa: E402
from dynosam_amd.optimizer import Solver, set_tile_ordering  # noqa: E402
from oracle_binding import Oracle  # noqa: E402
from test_gpu_parity import object_tangent_mask, gauge_split, lm_params, rel  # noqa: E402


def make(name, **kw):
    g, v, _ = synth.generate(name, **kw)
    s = Solver(0)
    s.set_graph(g)
    s.set_values(v)
    return g, v, s


def tr(e):
    return (e["outer_iteration"], f"{e['lam']:.0e}", e["solved"], e["accepted"], f"{e['current_error']:.12e}",
            f"{e['new_error']:.12e}", f"{e['model_fidelity']:.4e}")


print("=== A: LLWorld T2 free runs", flush=True)
g, v, s = make("T2", formulation=1)
sg = s.optimize()
o = Oracle(g, v)
so = o.optimize()
print("gpu", sg.iterations, sg.inner_iterations, "oracle", so.iterations, so.inner_iterations)
for a, b in zip(s.trace(), o.trace()):
    print("G", tr(a))
    print("O", tr(b))

for name, iters in (("T2", 8), ("C1", 6)):
    print(f"=== B: LLWorld {name} conditioned", flush=True)
    g, v, s = make(name, formulation=1)
    o = Oracle(g, v)
    mt, _ = object_tangent_mask(v)
    lam = 1e-5
    for it in range(iters):
        start = s.values_data()
        o.set_values_data(start)
        o.reset(lm_params(lam))
        s.reset(lm_params(lam))
        sg, so = s.iterate(), o.iterate()
        after = s.values_data()
        tg, to = s.trace(), o.trace()
        same = (sg.iterations, sg.inner_iterations) == (so.iterations, so.inner_iterations)
        print(it, "same" if same else "DIFF", [tr(e) for e in tg], [tr(e) for e in to])
        if not same:
            for mult in (1, 10, 100, 1000):
                lj = next(tg[i]["lam"] for i in range(min(len(tg), len(to))) if tg[i]["accepted"] != to[i]["accepted"]
                          or tg[i]["solved"] != to[i]["solved"]) * mult
                s.set_values(v.with_data(start))
                okg, dg = s.solve_delta(lj)
                o.set_values_data(start)
                oko, do = o.solve_damped(lj)
                fr, nd = gauge_split(v, dg, do)
                print("   lam", lj, "ok", okg, oko, "nonobj rel", rel(dg[~mt], do[~mt]), "obj rel", rel(dg[mt], do[mt]),
                      "off-gauge frac", fr, "diff", nd, "|d_obj|", np.linalg.norm(do[mt]))
            s.set_values(v.with_data(after))
        lam = sg.final_lambda

print("=== C: C2 conditioned late iterations", flush=True)
g, v, s = make("C2")
set_tile_ordering(2)
c = Solver(0)
c.set_graph(g)
c.set_values(v)
set_tile_ordering(-1)
o = Oracle(g, v, threads=16)
s.reset()
o.reset()
kinds = v.kinds
keys = v.keys
off = v._offsets()
for it in range(15):
    start = s.values_data()
    o.set_values_data(start)
    lam_before = s.trace()[-1]["lam"] if s.trace() else 1e-5
    sg, so = s.iterate(), o.iterate()
    tg = s.trace()
    c.set_values(v.with_data(start))
    c.reset(lm_params(tg[-1]["lam"] if tg[-1]["accepted"] else tg[-1]["lam"]))
    gv, ov = s.values_data(), o.values_data()
    d = gv - ov
    parts = {}
    for i, k in enumerate(keys):
        ch = chr(int(k) >> 56)
        parts.setdefault(ch, [0.0, 0.0])
        seg = slice(off[i], off[i + 1])
        parts[ch][0] += float(d[seg] @ d[seg])
        parts[ch][1] += float(ov[seg] @ ov[seg])
    worst = int(np.argmax(np.abs(d)))
    wi = int(np.searchsorted(off, worst, side="right") - 1)
    print(it, "lam", tg[-1]["lam"], "rel", rel(gv, ov), {k: f"{np.sqrt(a):.2e}/{np.sqrt(b):.2e}" for k, (a, b) in parts.items()},
          "worst key", chr(int(keys[wi]) >> 56), int(keys[wi]) & ((1 << 48) - 1), f"{d[worst]:.2e}", flush=True)
    # the GPU step from the same state with another tile ordering (pure reordering)
    if it >= 10:
        for lamx in (tg[0]["lam"],):
            s2 = Solver(0)
            okg, dg = s.solve_delta(lamx) if False else (None, None)
        o2 = Oracle(g, v, threads=16)
        o2.set_values_data(start)
        s.set_values(v.with_data(start))
        lj = tg[0]["lam"]
        okg, dg = s.solve_delta(lj)
        okc, dc = c.solve_delta(lj)
        oko, do = o2.solve_damped(lj)
        print("    step at lam", lj, "gpu-oracle", rel(dg, do), "gpu(leaf2)-gpu", rel(dc, dg), "gpu(leaf2)-oracle",
              rel(dc, do), "|step|", np.linalg.norm(do), flush=True)
        s.set_values(v.with_data(gv))
