"""Host planner of the tile Cholesky (dynosam_amd/csrc/tiles.cpp), checked
without a GPU.

The schedule exported by dynohip_plan_schedule is replayed task by task in
numpy: the panel and update semantics of k_tasks / k_back
(csrc/tilechol.hip) and the slot lookup of the assembly (tile_index in
csrc/kernels.hip). The replay checks three things:
  * no two tasks of one level conflict (write/write or read/write on a
    tile, a right-hand-side block or an output);
  * the assembly finds a slot for every nonzero 64x64 block (diagonal
    tiles stored full and symmetric, as k_gather_band writes them);
  * the replayed factor and solve reproduce numpy.linalg.solve on a random
    SPD matrix with the plan's block sparsity.
This covers frame order (the plain band), forced nested dissection and the
automatic choice.
"""
import numpy as np
import pytest

from dynosam_amd import synth
from dynosam_amd.optimizer import plan_schedule, set_tile_ordering

T = 64


def random_reduced(sched, rng):
    """SPD matrix with nonzero 6x6 blocks exactly at the plan's pose pairs,
    padded to NT*64 with the identity (k_tile_pad)."""
    n_red = 6 * sched["n_pose"]
    NT = sched["n_tiles"]
    M = np.zeros((NT * T, NT * T))
    for a, b in zip(sched["red_a"], sched["red_b"]):
        blk = rng.standard_normal((6, 6)) * 0.3
        if a == b:
            blk = blk @ blk.T
        M[6 * a:6 * a + 6, 6 * b:6 * b + 6] = blk
        if a != b:
            M[6 * b:6 * b + 6, 6 * a:6 * a + 6] = blk.T
    d = np.abs(M).sum(axis=1) + 1.0
    M[np.arange(n_red), np.arange(n_red)] = d[:n_red]
    M[np.arange(n_red, NT * T), np.arange(n_red, NT * T)] = 1.0
    return M


def slot_of(sched, i, j):
    lo, hi = sched["row_start"][i], sched["row_start"][i + 1]
    cols = sched["row_col"][lo:hi]
    k = np.searchsorted(cols, j)
    assert k < len(cols) and cols[k] == j, f"no slot for tile ({i}, {j})"
    return int(sched["row_slot"][lo + k])


def assemble(sched, M):
    NT, pos = sched["n_tiles"], sched["tile_pos"]
    slots = np.zeros((sched["n_slots"], T, T))
    for ti in range(NT):
        for tj in range(ti + 1):
            blk = M[ti * T:(ti + 1) * T, tj * T:(tj + 1) * T]
            if not blk.any():
                continue
            if ti == tj:
                slots[slot_of(sched, ti, ti)] += blk     # diagonal tiles are stored symmetric
            elif pos[ti] >= pos[tj]:
                slots[slot_of(sched, ti, tj)] += blk
            else:
                slots[slot_of(sched, tj, ti)] += blk.T
    return slots


def replay(sched, M, rhs):
    NT = sched["n_tiles"]
    slots = assemble(sched, M)
    r = rhs.reshape(NT, T)
    contrib = np.zeros((sched["n_slots"], T))
    y = np.zeros((NT, T))
    Linv = np.zeros((NT, T, T))
    ft, fl, pairs = sched["ftask"], sched["flevel"], sched["pairs"]
    rs, rc, rsl = sched["row_start"], sched["row_col"], sched["row_slot"]

    def psum(beg, end):
        return sum((slots[pairs[e][0]] @ slots[pairs[e][1]].T for e in range(beg, end)), np.zeros((T, T)))

    def pslots(beg, end):
        return {("s", int(v)) for e in range(beg, end) for v in pairs[e]}

    for lv in range(len(fl) - 1):
        reads, writes = [], []
        for q in range(fl[lv], fl[lv + 1]):
            kind, k, i, dst, diag, pdb, pde, pob, poe, _ = (int(v) for v in ft[q])
            if kind == 1:
                reads.append(pslots(pob, poe) | {("s", dst)})
                writes.append({("s", dst)})
                continue
            rd = {("s", diag)} | pslots(pdb, pde)
            rd |= {("c", int(rsl[e])) for e in range(rs[k], rs[k + 1]) if rc[e] != k}
            if i != k:
                rd |= {("s", dst)} | pslots(pob, poe)
                writes.append({("s", dst), ("c", dst)})
            else:
                writes.append({("L", k), ("y", k)})
            reads.append(rd)
        for a in range(len(writes)):
            for b in range(len(writes)):
                if a != b:
                    bad = writes[a] & (reads[b] | writes[b])
                    assert not bad, f"level {lv}: conflict {bad}"
        for q in range(fl[lv], fl[lv + 1]):
            kind, k, i, dst, diag, pdb, pde, pob, poe, _ = (int(v) for v in ft[q])
            if kind == 1:
                slots[dst] -= psum(pob, poe)
                continue
            for e in range(pdb, pde):
                assert pairs[e][0] == pairs[e][1]
            A = slots[diag] - psum(pdb, pde)
            assert np.allclose(A, A.T, rtol=0, atol=1e-9 * np.abs(A).max())
            Li = np.linalg.inv(np.linalg.cholesky(A))
            rk = r[k] - sum((contrib[rsl[e]] for e in range(rs[k], rs[k + 1]) if rc[e] != k), np.zeros(T))
            yk = Li @ rk
            if i == k:
                Linv[k] = Li
                y[k] = yk
            else:
                L = (slots[dst] - psum(pob, poe)) @ Li.T
                slots[dst] = L
                contrib[dst] = L @ yk
    x = np.full((NT, T), np.nan)
    bt, bl, be = sched["btask"], sched["blevel"], sched["bent"]
    for lv in range(len(bl) - 1):
        ks = [int(bt[q][0]) for q in range(bl[lv], bl[lv + 1])]
        for q in range(bl[lv], bl[lv + 1]):
            k, beg, end, _ = (int(v) for v in bt[q])
            s = y[k].copy()
            for e in range(beg, end):
                sl, row = int(be[e][0]), int(be[e][1])
                assert row not in ks, "backward level reads a tile it solves"
                assert np.isfinite(x[row]).all(), "backward reads an unsolved tile"
                s -= slots[sl].T @ x[row]
            x[k] = Linv[k].T @ s
    return x.reshape(-1)


def schedule_for(name, leaf, **kw):
    graph, values, _ = synth.generate(name, **kw)
    set_tile_ordering(leaf)
    try:
        return plan_schedule(graph, values)
    finally:
        set_tile_ordering(-1)


@pytest.mark.parametrize("name,leaf", [("T2", 0), ("T2", 2), ("C1", 0), ("C1", 4), ("C1", -1),
                                       ("C2", 0), ("C2", 6), ("C2", -1)])
def test_schedule_replay_solves(name, leaf):
    sched = schedule_for(name, leaf)
    if leaf >= 0:
        assert sched["nd_leaf"] == leaf
    rng = np.random.default_rng(7)
    M = random_reduced(sched, rng)
    rhs = rng.standard_normal(M.shape[0])
    x = replay(sched, M, rhs)
    ref = np.linalg.solve(M, rhs)
    assert np.allclose(x, ref, rtol=1e-9, atol=1e-10)


def test_large_system_grouped_updates_replay_solves():
    """A system of >= 128 tiles (tiles.cpp kUpdGroupTiles): its update tasks
    take the contributions of two ready levels each. The replay still solves
    exactly, and the grouping leaves fewer update tasks than ready levels."""
    sched = schedule_for(None, 16, frames=360, objects=3, static_landmarks=6000, dyn_slots=4)
    ft = sched["ftask"].reshape(-1, 10)
    assert sched["n_tiles"] >= 128, sched["n_tiles"]
    rng = np.random.default_rng(9)
    M = random_reduced(sched, rng)
    rhs = rng.standard_normal(M.shape[0])
    x = replay(sched, M, rhs)
    assert np.allclose(x, np.linalg.solve(M, rhs), rtol=1e-9, atol=1e-10)
    upd = ft[ft[:, 0] == 1]
    assert (upd[:, 8] - upd[:, 7]).max() >= 2   # some update applies contributions of two levels


def test_llworld_schedule_replay():
    sched = schedule_for("C1", 4, formulation=1)
    rng = np.random.default_rng(3)
    M = random_reduced(sched, rng)
    rhs = rng.standard_normal(M.shape[0])
    assert np.allclose(replay(sched, M, rhs), np.linalg.solve(M, rhs), rtol=1e-9, atol=1e-10)


def test_nested_dissection_shortens_critical_path():
    band = schedule_for("C2", 0)
    nd = schedule_for("C2", 6)
    assert band["n_flevel"] - 1 == band["n_tiles"]   # one column per level
    assert nd["n_flevel"] < band["n_flevel"] // 2
    assert sorted(nd["tile_pos"]) == list(range(nd["n_tiles"]))


def queue_is_topological(ftask, fdep_start, fdep, queue):
    """Every dependency of a task (the writer of the awaited write of a slot,
    writes counted in schedule order) comes earlier in the dataflow queue."""
    n = ftask.shape[0]
    assert sorted(queue.tolist()) == list(range(n))
    pos = np.empty(n, dtype=np.int64)
    pos[queue] = np.arange(n)
    writer, cnt = {}, {}
    for q in range(n):
        if ftask[q, 0] == 1 or ftask[q, 1] != ftask[q, 2]:
            c = cnt.get(int(ftask[q, 3]), 0) + 1
            cnt[int(ftask[q, 3])] = c
            writer[(int(ftask[q, 3]), c)] = q
    for q in range(n):
        for j in range(fdep_start[q], fdep_start[q + 1]):
            assert pos[writer[(int(fdep[j, 0]), int(fdep[j, 1]))]] < pos[q]


@pytest.mark.parametrize("name", ["C1", "C2"])
def test_dataflow_queue_order_is_topological(name):
    """tiles.cpp queue_order: the list-scheduled queue of k_factor_persist is
    a permutation of the tasks in a topological order of the dataflow
    dependencies (the launch's deadlock freedom), and not the level order."""
    from dynosam_amd.optimizer import plan_export
    g, v, _ = synth.generate(name)
    ft = plan_export(g, v, "ftask").reshape(-1, 10)
    fs = plan_export(g, v, "fdep_start")
    fd = plan_export(g, v, "fdep").reshape(-1, 2)
    qu = plan_export(g, v, "fqueue")
    queue_is_topological(ft, fs, fd, qu)
    if name == "C2":
        assert not np.array_equal(qu, np.arange(ft.shape[0]))


def test_partitioned_queue_orders_are_topological():
    from dynosam_amd.optimizer import plan_export
    g, v, _ = synth.generate("C2")
    for nranks in (2, 4):
        for rank in range(nranks):
            nph = len(plan_export(g, v, "phases", nranks=nranks, rank=rank)) // 2
            for pre in [""] + [f"phase{k}_" for k in range(nph)]:
                ft = plan_export(g, v, pre + "ftask", nranks=nranks, rank=rank).reshape(-1, 10)
                fs = plan_export(g, v, pre + "fdep_start", nranks=nranks, rank=rank)
                fd = plan_export(g, v, pre + "fdep", nranks=nranks, rank=rank).reshape(-1, 2)
                qu = plan_export(g, v, pre + "fqueue", nranks=nranks, rank=rank)
                queue_is_topological(ft, fs, fd, qu)
