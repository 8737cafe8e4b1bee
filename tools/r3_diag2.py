"""C2 late LM iterations: GPU vs oracle step, reorder control and backward
errors of both solves (test infrastructure)."""
import os
import sys

import numpy as np
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from dynosam_amd import _abi, synth  # noqa: E402
from dynosam_amd.optimizer import Solver, set_tile_ordering  # noqa: E402
from oracle_binding import Oracle  # noqa: E402


def rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def sparse_system(graph, values, lin):
    """A (whitened, reweighted J) and b from a dynohip/oracle linearize() buffer"""
    tw = np.where(values.kinds == _abi.POSE3, 6, 3)
    toff = np.concatenate([[0], np.cumsum(tw)])
    idx = {int(k): i for i, k in enumerate(values.keys)}
    rows, cols, vals, b = [], [], [], []
    o = 0
    r0 = 0
    arr = graph.arrays()
    for t, name in enumerate(_abi.FACTOR_TYPES):
        keys = arr[name][0]
        n, nk = keys.shape
        if n == 0:
            continue
        d = _abi.FACTOR_DIM[t]
        vi = np.vectorize(lambda k: idx[int(k)])(keys)
        widths = tw[vi[0]]
        ncol = int(widths.sum())
        blk = lin[o:o + n * d * (ncol + 1)].reshape(n, d, ncol + 1)
        o += n * d * (ncol + 1)
        c = 0
        for sl in range(nk):
            w = int(widths[sl])
            base = toff[vi[:, sl]]
            for q in range(w):
                rr = (r0 + np.arange(n)[:, None] * d + np.arange(d)[None, :]).ravel()
                rows.append(rr)
                cols.append(np.repeat(base + q, d))
                vals.append(blk[:, :, c + q].ravel())
            c += w
        b.append(blk[:, :, ncol].ravel())
        r0 += n * d
    A = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(r0, toff[-1]))
    return A, np.concatenate(b)


def bwd(A, b, lam, x):
    """normwise backward error of (A^T A + lam I) x = A^T b"""
    r = A.T @ (A @ x) + lam * x - A.T @ b
    nH = sp.linalg.norm(A.T @ A, ord=1) + lam
    return float(np.linalg.norm(r, 1) / (nH * np.linalg.norm(x, 1) + np.linalg.norm(A.T @ b, 1)))


def main():
    g, v, _ = synth.generate("C2")
    s = Solver(0)
    s.set_graph(g)
    s.set_values(v)
    p = Solver(0)
    p.set_graph(g)
    p.set_values(v)
    set_tile_ordering(0)
    c = Solver(0)
    c.set_graph(g)
    c.set_values(v)
    set_tile_ordering(-1)
    o = Oracle(g, v, threads=16)
    s.reset()
    o.reset()
    for it in range(15):
        start = s.values_data()
        o.set_values_data(start)
        n0 = len(s.trace())
        sg, so = s.iterate(), o.iterate()
        tg = s.trace()[n0:]
        gv, ov = s.values_data(), o.values_data()
        print(it, [(e["lam"], e["accepted"]) for e in tg], (sg.iterations, sg.inner_iterations),
              (so.iterations, so.inner_iterations), "values rel", rel(gv, ov), flush=True)
        if it >= 9:
            lam = tg[-1]["lam"]
            p.set_values(v.with_data(start))
            c.set_values(v.with_data(start))
            okg, dg = p.solve_delta(lam)
            okc, dc = c.solve_delta(lam)
            chk = Oracle(g, v, threads=16)
            chk.set_values_data(start)
            oko, do = chk.solve_damped(lam)
            A, b = sparse_system(g, v, chk.linearize())
            print("   lam", lam, "ok", okg, okc, oko, "step rel gpu-oracle", rel(dg, do), "gpu(frame order)-gpu", rel(dc, dg),
                  "|step|", np.linalg.norm(do), "bwd err gpu", bwd(A, b, lam, dg), "gpu(frame)", bwd(A, b, lam, dc),
                  "oracle", bwd(A, b, lam, do), flush=True)


if __name__ == "__main__":
    main()
