"""Graphs beyond the synthetic generator's, for the plan and parity tests.

mixed_lone_graph: T2 with two static landmarks made ineligible for the
lone-point groups (plan.hpp LoneGroup): one gets a second PoseToPoint factor
to a pose it already sees, the other is observed from 11 poses (more than
kLoneMaxNb). The plan then keeps the CSR point gathers, the lone Y and the
per-point back-substitution for every lone point, and the groups for the
rest (lone_all_grouped = false)."""
import numpy as np

from dynosam_amd import synth
from dynosam_amd.graph import NonlinearFactorGraph


def mixed_lone_graph():
    g, v, gt = synth.generate("T2")
    a = {t: list(x) for t, x in g.arrays().items()}
    keys, meas, sig, hub = a["pose_to_point"]
    pts = keys[:, 1]
    static = [p for p in np.unique(pts) if (int(p) >> 56) == ord("l")] or list(np.unique(pts))
    # the static landmark with the most observations, and another one
    counts = {int(p): int((pts == p).sum()) for p in static}
    p_dup, p_wide = sorted(counts, key=lambda p: (-counts[p], p))[:2]
    rows_k, rows_m = [], []
    i = int(np.flatnonzero(pts == np.uint64(p_dup))[0])
    rows_k.append(keys[i].copy())
    rows_m.append(meas[i] + 0.01)
    seen = set(int(x) for x in keys[pts == np.uint64(p_wide), 0])
    j = int(np.flatnonzero(pts == np.uint64(p_wide))[0])
    for pose in np.unique(keys[:, 0]):
        if len(seen) >= 11:
            break
        if int(pose) not in seen:
            seen.add(int(pose))
            rows_k.append(np.array([pose, p_wide], dtype=np.uint64))
            rows_m.append(meas[j])
    n = len(rows_k)
    a["pose_to_point"] = [np.concatenate([keys, np.array(rows_k, dtype=np.uint64)]),
                          np.concatenate([meas, np.array(rows_m)]),
                          np.concatenate([sig, np.repeat(sig[:1], n, axis=0)]),
                          np.concatenate([hub, np.repeat(hub[:1], n)])]
    return NonlinearFactorGraph.from_arrays({t: tuple(x) for t, x in a.items()}), v, gt, (p_dup, p_wide)
