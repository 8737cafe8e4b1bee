"""Replicated separator work of the partitioned solve.

For each graph and rank count: every rank's phase-0 factorisation flops
(its subtree and its interior columns' updates of separator tiles), the
phase-1 flops every rank repeats (the separator columns), and the exchanged
doubles per linear solve (the separator tiles and RHS rows). Flops are the
algorithmic tile counts the schedule builder uses: a diagonal factor T^3/3,
an off-diagonal panel T^3, an update pair 2 T^3 (T = 64). Host-only (plan
export). Usage: python tools/sep_flops.py [C2 NS C5]"""
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
                p0 = [task_flops(plan_export(g, v, "ftask", nr, r)) for r in range(nr)]
                p1 = task_flops(plan_export(g, v, "ftask1", nr, 0))
                ssr = plan_export(g, v, "sep_slot_ranges", nr, 0)
                str_ = plan_export(g, v, "sep_tile_ranges", nr, 0)
            except Exception as e:  # too short in time for that many ranks
                print(f"  {nr} ranks: no partition ({e})")
                continue
            ntile = int((ssr[1::2] - ssr[0::2]).sum())
            nrow = int((str_[1::2] - str_[0::2]).sum())
            xd = ntile * T * T + nrow * T
            print(f"  {nr} ranks: phase 0 per rank max {max(p0) / 1e9:.3f} min {min(p0) / 1e9:.3f} GFLOP,"
                  f" phase 1 (every rank) {p1 / 1e9:.3f} GFLOP = {p1 / (sum(p0) + p1):.1%} of the"
                  f" partitioned total, replicated {(nr - 1) * p1 / 1e9:.3f} GFLOP;"
                  f" exchange {ntile} tiles + {nrow} rows = {xd} doubles ({8 * xd / 1e6:.2f} MB)")


if __name__ == "__main__":
    main(sys.argv[1:] or ["C2", "NS", "C5"])
