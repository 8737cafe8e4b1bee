"""Where the GPU and oracle linearisations differ (per factor type, J vs b),
at C2 states along the LM run (test infrastructure)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from dynosam_amd import _abi, synth  # noqa: E402
from dynosam_amd.optimizer import Solver  # noqa: E402
from oracle_binding import Oracle  # noqa: E402

g, v, _ = synth.generate("C2")
s = Solver(0)
s.set_graph(g)
s.set_values(v)
p = Solver(0)
p.set_graph(g)
p.set_values(v)
s.reset()
tw = np.where(v.kinds == _abi.POSE3, 6, 3)
idx = {int(k): i for i, k in enumerate(v.keys)}
arr = g.arrays()
for it in range(15):
    start = s.values_data()
    if it in (0, 9, 13):
        p.set_values(v.with_data(start))
        lg = p.linearize()
        o = Oracle(g, v, threads=16)
        o.set_values_data(start)
        lo = o.linearize()
        off = 0
        for t, name in enumerate(_abi.FACTOR_TYPES):
            keys = arr[name][0]
            n = keys.shape[0]
            if n == 0:
                continue
            d = _abi.FACTOR_DIM[t]
            ncol = int(sum(tw[idx[int(k)]] for k in keys[0]))
            G = lg[off:off + n * d * (ncol + 1)].reshape(n, d, ncol + 1)
            O = lo[off:off + n * d * (ncol + 1)].reshape(n, d, ncol + 1)
            off += n * d * (ncol + 1)
            for part, sl in (("J", np.s_[:, :, :ncol]), ("b", np.s_[:, :, ncol])):
                a, b = G[sl], O[sl]
                dd = np.abs(a - b)
                cr = dd / np.maximum(np.abs(b), 1e-300)
                nz = np.abs(b) > 1e-300
                if not nz.any():
                    continue
                rowscale = np.max(np.abs(O[:, :, :ncol]), axis=(1, 2))
                scaled = (dd.reshape(n, -1).max(axis=1) / np.maximum(rowscale, 1e-300))
                w = int(np.argmax(scaled))
                print(it, name, part, "componentwise rel p50 %.1e p99 %.1e max %.1e" % (
                    np.percentile(cr[nz], 50), np.percentile(cr[nz], 99), cr[nz].max()),
                    "| per-factor max|diff|/max|J| p99 %.1e max %.1e (factor %d)" % (
                        np.percentile(scaled, 99), scaled.max(), w), flush=True)
            if name in ("pose_to_point", "landmark_motion_ternary", "between", "prior"):
                w = int(np.argmax(np.abs(G - O).reshape(n, -1).max(axis=1) / np.maximum(np.max(np.abs(O), axis=(1, 2)), 1e-300)))
                print("   worst factor", w, "keys", [hex(int(k)) for k in keys[w]], "\n   gpu b", G[w, :, ncol],
                      "\n   orc b", O[w, :, ncol], "\n   gpu J0", G[w, 0, :ncol], "\n   orc J0", O[w, 0, :ncol], flush=True)
    s.iterate()
