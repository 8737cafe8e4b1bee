"""Separator work of the partitioned solve.

For each graph and rank count: every rank's phase-0 factorisation flops
(its subtree and its interior columns' updates of separator tiles) and its
separator-phase flops (one node per depth: the node's panels and own-tile
updates, which every rank of the node's group runs, plus, on the group's
leader only, the node's updates of the separators above), the share of the
heaviest rank's work that other ranks repeat (its nodes' group-wide tasks),
and the exchanged doubles per linear solve (each separator's tiles and RHS
rows once, in one all-reduce per depth). Flops are the algorithmic tile
counts the schedule builder uses: a diagonal factor T^3/3, an off-diagonal
panel T^3, an update pair 2 T^3 (T = 64). Host-only (plan export).
Usage: python tools/sep_flops.py [C2 NS C5]"""
import sys

import numpy as np

sys.path.insert(0, ".")
from dynosam_amd import synth  # noqa: E402
from dynosam_amd.optimizer import plan_export  # noqa: E402

T = 64
T3 = float(T) ** 3


def task_flops(ft):
    if ft.size == 0:
        return 0.0
    kind, k, i = ft[:, 0], ft[:, 1], ft[:, 2]
    pd = ft[:, 6] - ft[:, 5]
    po = ft[:, 8] - ft[:, 7]
    panel = kind == 0
    diag = panel & (k == i)
    f = np.where(diag, T3 / 3, 0.0) + np.where(panel & ~diag, T3, 0.0)
    # a column's panels share the diagonal's pending pairs: counted once, at the diagonal
    f = f + np.where(diag, 2 * T3 * pd, 0.0) + 2 * T3 * po
    return float(f.sum())


def main(names):
    for name in names:
        g, v, _ = synth.generate(name)
        single = task_flops(plan_export(g, v, "ftask", 1, 0))
        print(f"{name}: single-handle factorisation {single / 1e9:.3f} GFLOP")
        for nr in (2, 4, 8):
            try:
                rows = []
                for r in range(nr):
                    p0 = task_flops(plan_export(g, v, "ftask", nr, r))
                    ph = plan_export(g, v, "phases", nr, r).reshape(-1, 2)
                    sep = [task_flops(plan_export(g, v, f"phase{k}_ftask", nr, r)) for k in range(len(ph))]
                    rows.append((p0, sep, ph))
                nodes = plan_export(g, v, "sep_nodes", nr, 0).reshape(-1, 5)
                xd = 0
                for k in range(len(rows[0][2])):
                    xs = plan_export(g, v, f"phase{k}_xslot", nr, 0)
                    xt = plan_export(g, v, f"phase{k}_xtile", nr, 0)
                    xd += int((xs[1::2] - xs[0::2]).sum()) * T * T + int((xt[1::2] - xt[0::2]).sum()) * T
            except Exception as e:  # too short in time for that many ranks
                print(f"  {nr} ranks: no partition ({e})")
                continue
            tot = [p0 + sum(sep) for p0, sep, _ in rows]
            h = int(np.argmax(tot))
            p0, sep, ph = rows[h]
            # the heaviest rank's node work that its group's other ranks repeat:
            # a non-leader's whole node phase; a leader's phase minus its
            # leader-only updates (the smallest member phase of the node)
            rep = 0.0
            for k, (node, leader) in enumerate(ph):
                if nodes[node][1] <= 1:
                    continue
                member = min(rows[r][1][k] for r in range(nr) if rows[r][2][k][0] == node)
                rep += member
            work_all = sum(tot)
            print(f"  {nr} ranks: heaviest rank {h}: phase 0 {p0 / 1e9:.3f} + separator phases "
                  f"{sum(sep) / 1e9:.3f} GFLOP ({' + '.join(f'{x / 1e9:.3f}' for x in sep)}, deepest first); "
                  f"lightest total {min(tot) / 1e9:.3f}; repeated by other ranks {rep / 1e9:.3f} GFLOP = "
                  f"{rep / tot[h]:.1%} of the heaviest rank's work; all ranks {work_all / 1e9:.3f} GFLOP "
                  f"(flops bound on efficiency {single / (nr * tot[h]):.2f}); exchange {xd} doubles "
                  f"({8 * xd / 1e6:.2f} MB) in {len(ph)} all-reduces")


if __name__ == "__main__":
    main(sys.argv[1:] or ["C2", "NS", "C5"])
