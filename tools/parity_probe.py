"""Measurements behind the hardened parity tests (round 6): the quantities
the tests bound, printed per case so the bounds can be set from data with a
stated margin. Needs the GPU. usage: python tools/parity_probe.py CASE...
cases: llworld_c2 (per-iteration, conditioned, against the oracle in both
summation orders), ns_free (end points: GPU, oracle forward / reversed
orders, exact-step run), c2_libm (free runs: GPU, oracle, glibc-trig
oracle, exact-step run), windows (configs[3]: every window's full
conditioned run and free-run end)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from dynosam_amd.optimizer import Solver  # noqa: E402
from oracle_binding import Oracle  # noqa: E402
import test_gpu_parity as T  # noqa: E402


def llworld_c2(iters=12):
    g, v, _, s = T.make("C2", formulation=1)
    A = Oracle(g, v, threads=T.cores())
    B = Oracle(g, v, threads=T.cores(), reverse_sums=True)
    E = Oracle(g, v, threads=T.cores(), solve_ld=True)   # exact steps (x87 extended precision)
    m = T.gauge_mask(v)
    lam = 1e-5
    rows = []
    for it in range(iters):
        start = s.values_data()
        for o in (A, B, E):
            o.set_values_data(start)
            o.reset(T.lm_params(lam))
        s.reset(T.lm_params(lam))
        sg, sa, sb, se = s.iterate(), A.iterate(), B.iterate(), E.iterate()
        tg, ta, tb, te = s.trace(), A.trace(), B.trace(), E.trace()
        key = lambda t: [(e["lam"], e["solved"], e["accepted"]) for e in t]
        vg, va, vb, ve = s.values_data(), A.values_data(), B.values_data(), E.values_data()
        mo = lambda x: T.llworld_motions(v, x)
        row = {"it": it, "lam": lam, "counts": [(x.iterations, x.inner_iterations) for x in (sg, sa, sb)],
               "tries_gA": key(tg) == key(ta), "tries_gB": key(tg) == key(tb), "tries_AB": key(ta) == key(tb),
               "nonobj_gA": T.rel(vg[m], va[m]), "nonobj_gB": T.rel(vg[m], vb[m]), "nonobj_AB": T.rel(va[m], vb[m]),
               "mot_gA": T.rel(mo(vg), mo(va)), "mot_gB": T.rel(mo(vg), mo(vb)), "mot_AB": T.rel(mo(va), mo(vb)),
               "tries_gE": key(tg) == key(te), "tries_AE": key(ta) == key(te), "tries_BE": key(tb) == key(te),
               "nonobj_gE": T.rel(vg[m], ve[m]), "nonobj_AE": T.rel(va[m], ve[m]),
               "mot_gE": T.rel(mo(vg), mo(ve)), "mot_AE": T.rel(mo(va), mo(ve)), "mot_BE": T.rel(mo(vb), mo(ve)),
               "trace_g": key(tg), "trace_A": key(ta), "trace_E": key(te),
               "moved": float(np.linalg.norm(vg - start))}
        rows.append(row)
        print(json.dumps(row), flush=True)
        lam = sg.final_lambda
    return rows


def ns_free():
    g, v, _, s = T.make("NS")
    sg = s.optimize()
    vg = s.values_data()
    out = {"gpu": (sg.iterations, sg.inner_iterations)}
    ends = {}
    for name, kw in (("fw", {}), ("rv", {"reverse_sums": True})):
        o = Oracle(g, v, threads=T.cores(), **kw)
        so = o.optimize()
        ends[name] = o.values_data()
        out[name] = (so.iterations, so.inner_iterations)
    ex = np.load(os.path.join(ROOT, "tests", "golden", "ns_exact_lm.npz"))
    ends["exact"] = ex["values"]
    for a in ends:
        out[f"gpu_{a}"] = T.rel(vg, ends[a])
    out["fw_rv"] = T.rel(ends["fw"], ends["rv"])
    out["fw_exact"] = T.rel(ends["fw"], ends["exact"])
    out["rv_exact"] = T.rel(ends["rv"], ends["exact"])
    print(json.dumps(out), flush=True)


def c2_libm():
    g, v, _, s = T.make("C2")
    sg = s.optimize()
    vg = s.values_data()
    out = {"gpu": (sg.iterations, sg.inner_iterations)}
    ends = {}
    for name, kw in (("oracle", {}), ("libm", {"libm": True}), ("libm_rv", {"libm": True, "reverse_sums": True}),
                     ("exact", {"solve_ld": True}), ("libm_exact", {"libm": True, "solve_ld": True})):
        o = Oracle(g, v, threads=T.cores(), **kw)
        so = o.optimize()
        ends[name] = o.values_data()
        out[name] = (so.iterations, so.inner_iterations)
    names = list(ends)
    for a in names:
        out[f"gpu_{a}"] = T.rel(vg, ends[a])
    for i, a in enumerate(names):
        for b in names[i + 1:]:
            out[f"{a}_{b}"] = T.rel(ends[a], ends[b])
    print(json.dumps(out), flush=True)


def windows():
    import test_windows as W
    for w in range(W.N_WINDOWS_C4):
        g, v = W._c4_window(w)
        s = Solver(0)
        s.set_graph(g)
        s.set_values(v)
        sg = s.optimize()
        n = sg.iterations
        vg_free = s.values_data()
        o = Oracle(g, v, threads=T.cores())
        so = o.optimize()
        free = {"counts": [(sg.iterations, sg.inner_iterations), (so.iterations, so.inner_iterations)],
                "err_rel": abs(sg.final_error - so.final_error) / so.final_error,
                "values_rel": T.rel(vg_free, o.values_data())}
        s.set_values(v)
        s.reset()
        lam, worst, same = 1e-5, 0.0, True
        for it in range(n):
            start = s.values_data()
            o.set_values_data(start)
            o.reset(T.lm_params(lam))
            s.reset(T.lm_params(lam))
            a, b = s.iterate(), o.iterate()
            same &= (a.iterations, a.inner_iterations) == (b.iterations, b.inner_iterations)
            worst = max(worst, T.rel(s.values_data(), o.values_data()))
            lam = a.final_lambda
        print(json.dumps({"window": w, "iterations": n, "conditioned_worst": worst, "same_counts": same,
                          "free": free}), flush=True)


if __name__ == "__main__":
    for case in sys.argv[1:]:
        print("==", case, flush=True)
        globals()[case]()
