"""Structural zeros inside the 64x64 tiles of the reduced-system Cholesky.

The tile DAG (tiles.cpp) issues every MFMA of a 64x64 tile product, fill
included. This tool takes the pose-level pattern of the reduced system
(dynohip_plan_schedule: red_a / red_b, tile_pos), runs the symbolic
Cholesky at the 6x6 pose-block level in the schedule's elimination order
(tiles by position, poses in natural order inside a tile; a pose straddling
two tiles takes the earlier one's position), and counts, per stored tile,
which of its 4 x 4 sub-blocks of 16 x 16 hold a structural nonzero. It
then prices the factorisation's tasks at 16 x 16 x 16 sub-block granularity
(an update's product L(i,c) L(j,c)^T only over k-blocks where both
operands' rows are nonzero) against the full 64^3 tile products.
Host-only. usage: python tools/tile_fill.py [C2 NS]"""
import sys

import numpy as np

sys.path.insert(0, ".")
from dynosam_amd import synth  # noqa: E402
from dynosam_amd.optimizer import plan_schedule  # noqa: E402

T = 64
B = 16


def analyse(name):
    g, v, _ = synth.generate(name)
    sc = plan_schedule(g, v)
    n_pose, NT = sc["n_pose"], sc["n_tiles"]
    tpos = sc["tile_pos"]
    # pose elimination key: (position of its first dimension's tile, pose)
    key = np.array([tpos[(6 * p) // T] * 100000 + p for p in range(n_pose)])
    order = np.argsort(key)
    rank = np.empty(n_pose, dtype=np.int64)
    rank[order] = np.arange(n_pose)
    adj = [set() for _ in range(n_pose)]
    for a, b in zip(sc["red_a"], sc["red_b"]):
        if a != b:
            ra, rb = rank[a], rank[b]
            lo, hi = min(ra, rb), max(ra, rb)
            adj[lo].add(hi)
    # symbolic factorisation in rank space (elimination tree merge)
    struct = [None] * n_pose
    parent_children = [[] for _ in range(n_pose)]
    for j in range(n_pose):
        s = set(adj[j])
        for c in parent_children[j]:
            s |= struct[c]
        s.discard(j)
        struct[j] = s
        if s:
            parent_children[min(s)].append(j)
    # nonzero 16x16 sub-blocks per (row tile, col tile): dims of pose p are 6p..6p+5
    sub = {}
    for j in range(n_pose):
        pj = order[j]
        cols = range(6 * pj, 6 * pj + 6)
        rows_p = [order[i] for i in struct[j]] + [pj]
        for pi in rows_p:
            for rr in range(6 * pi, 6 * pi + 6):
                for cc in cols:
                    ti, tc = rr // T, cc // T
                    # stored tile (row tile, col tile) by elimination position
                    if tpos[ti] < tpos[tc]:
                        ti, tc, rr, cc = tc, ti, cc, rr
                    m = sub.setdefault((ti, tc), np.zeros((4, 4), dtype=bool))
                    m[(rr % T) // B, (cc % T) // B] = True
    full = occ = 0
    for m in sub.values():
        full += 16
        occ += int(m.sum())
    # price the update pairs: every (i, c) and (j, c) stored below the diagonal of column c
    cols = {}
    for (ti, tc) in sub:
        if ti != tc:
            cols.setdefault(tc, []).append(ti)
    upd_full = upd_sub = 0
    for tc, rows in cols.items():
        for x in range(len(rows)):
            for y in range(x + 1):
                mi, mj = sub[(rows[x], tc)], sub[(rows[y], tc)]
                upd_full += 64
                upd_sub += int((mi[:, None, :] & mj[None, :, :]).sum())
    print(f"{name}: {len(sub)} stored tiles touched by the pose pattern, 16x16 sub-blocks nonzero "
          f"{occ}/{full} = {occ / full:.1%}; update products at 16^3 granularity {upd_sub}/{upd_full} = "
          f"{upd_sub / max(upd_full, 1):.1%} of the full tile products")


if __name__ == "__main__":
    for nm in sys.argv[1:] or ["C2", "NS"]:
        analyse(nm)
