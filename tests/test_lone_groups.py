"""Lone-point groups of the plan (plan.hpp LoneGroup): the
static landmarks whose Schur contributions one workgroup per group sums.
Checked on the host against the graph itself (no GPU): which lone points are
eligible, that every eligible point is in exactly one group, that a group's
points share its neighbour-pose list, the device block layout (points,
first edges, neighbour poses, PoseToPoint record offsets) and the near-equal
split of a list into groups of at most lone_cap(m) points."""
import numpy as np
import pytest

from dynosam_amd import synth
from dynosam_amd.optimizer import plan_export
from graphs_extra import mixed_lone_graph

# plan.hpp: kLoneMaxNb, kLoneSub, the header offsets and kLoneBlk
MAX_NB, SUB = 10, 32
HDR_PT, HDR_E0, HDR_POSE = 4, 4 + SUB, 4 + 2 * SUB
HDR_REC = HDR_POSE + MAX_NB
BLK = (HDR_REC + 256 + 3) // 4 * 4


def lone_cap(m):
    """points per block: a lane per (point, neighbour) in four 64-lane waves"""
    return min(4 * (64 // m), SUB)


@pytest.fixture(scope="module", params=[("T2", {}), ("T2", {"formulation": 1}), ("C1", {}), ("mixed", {})],
                ids=["T2", "T2-LLWorld", "C1", "T2-mixed"])
def plan(request):
    name, kw = request.param
    if name == "mixed":   # two lone points not eligible: lone_all_grouped = false
        g, v, _, _ = mixed_lone_graph()
    else:
        g, v, _ = synth.generate(name, **kw)
    ex = {k: plan_export(g, v, k) for k in ("lone_info", "lone_blk", "lgroup", "lone_pose", "pt_edges",
                                            "edge_pose", "comp_starts", "type_rec", "type_idx0", "type_idx1",
                                            "type_idx4")}
    return ex


def eligible_points(ex):
    all_grouped, ngroups, max_m, p_lone, n_pt = ex["lone_info"]
    pes, ep = ex["pt_edges"], ex["edge_pose"]
    idx0 = ex["type_idx0"].reshape(-1, 2)            # (pose, point)
    refs = {}
    for i, (pose, pt) in enumerate(idx0):
        refs.setdefault(int(pt), []).append((int(pose), i))
    other = set(ex["type_idx1"].reshape(-1, 3)[:, :2].ravel().tolist())   # ternary point slots
    other |= set(ex["type_idx4"].reshape(-1, 4)[:, :2].ravel().tolist())  # landmark-motion-pose point slots
    elig = {}
    for p in range(p_lone, n_pt):
        m = int(pes[p + 1] - pes[p])
        r = refs.get(p, [])
        poses = sorted(x[0] for x in r)
        if p in other or not 1 <= m <= MAX_NB or len(r) != m or poses != ep[pes[p]:pes[p + 1]].tolist():
            continue
        elig[p] = dict(r)   # pose -> factor index
    return elig


def test_groups_cover_the_eligible_lone_points_once(plan):
    ex = plan
    all_grouped, ngroups, max_m, p_lone, n_pt = ex["lone_info"]
    elig = eligible_points(ex)
    blk = ex["lone_blk"].reshape(-1, BLK)
    assert blk.shape[0] == ngroups
    seen = [int(p) for g in range(ngroups) for p in blk[g, HDR_PT:HDR_PT + blk[g, 1]]]
    assert sorted(seen) == sorted(elig)
    assert len(seen) == len(set(seen))
    assert bool(all_grouped) == (len(elig) == n_pt - p_lone)
    assert ngroups == 0 or max_m == max(int(blk[g, 0]) for g in range(ngroups))


def test_group_blocks_match_the_graph(plan):
    ex = plan
    ngroups = int(ex["lone_info"][1])
    elig = eligible_points(ex)
    blk = ex["lone_blk"].reshape(-1, BLK)
    lg = ex["lgroup"].reshape(-1, 4)
    pes, ep, lp = ex["pt_edges"], ex["edge_pose"], ex["lone_pose"]
    base0, stride0 = (int(x) & 0xffffffff for x in ex["type_rec"][:2])
    outs = []
    for g in range(ngroups):
        m, npt = int(blk[g, 0]), int(blk[g, 1])
        assert (m, npt) == (int(lg[g, 0]), int(lg[g, 1]))
        assert 1 <= m <= MAX_NB and 1 <= npt <= lone_cap(m) and npt * m <= 256
        poses = lp[lg[g, 2]:lg[g, 2] + m].tolist()
        assert poses == sorted(poses)
        assert blk[g, HDR_POSE:HDR_POSE + m].tolist() == poses
        assert not blk[g, HDR_POSE + m:HDR_REC].any()
        outs.append(int(blk[g, 2]) & 0xffffffff)
        assert outs[-1] == int(lg[g, 3]) & 0xffffffff
        for u in range(npt):
            p = int(blk[g, HDR_PT + u])
            assert int(blk[g, HDR_E0 + u]) == pes[p]
            assert ep[pes[p]:pes[p] + m].tolist() == poses
            for a in range(m):
                rec = int(blk[g, HDR_REC + m * u + a]) & 0xffffffff
                assert rec == base0 + stride0 * elig[p][poses[a]]
        assert not blk[g, HDR_PT + npt:HDR_PT + SUB].any()   # unused member slots are zero
    # partial areas: disjoint, in group order, m(m+1)/2 6x6 blocks + m gradients each
    for g in range(ngroups - 1):
        m = int(blk[g, 0])
        # per-try partial blocks and gradients, then the fused linearisation's
        # H area (42 m: J_a^T J_a and J_a^T b per neighbour)
        assert outs[g + 1] == outs[g] + 36 * (m * (m + 1) // 2) + 6 * m + 42 * m


def test_groups_split_lists_evenly_in_first_pose_order(plan):
    ex = plan
    ngroups = int(ex["lone_info"][1])
    blk = ex["lone_blk"].reshape(-1, BLK)
    lg = ex["lgroup"].reshape(-1, 4)
    lp = ex["lone_pose"]
    lists = [tuple(lp[lg[g, 2]:lg[g, 2] + lg[g, 0]].tolist()) for g in range(ngroups)]
    firsts = [l[0] for l in lists]
    assert firsts == sorted(firsts)
    sizes = {}
    for l, g in zip(lists, range(ngroups)):
        sizes.setdefault(l, []).append(int(blk[g, 1]))
    for l, s in sizes.items():
        assert max(s) - min(s) <= 1, l
        assert len(s) == -(-sum(s) // lone_cap(len(l))), l


def test_ineligible_lone_points_stay_out():
    g, v, _, (p_dup, p_wide) = mixed_lone_graph()
    info = plan_export(g, v, "lone_info")
    blk = plan_export(g, v, "lone_blk").reshape(-1, BLK)
    keys = np.asarray(v.keys)
    pes = plan_export(g, v, "pt_edges")
    assert info[0] == 0   # not every lone point grouped: CSR gathers, lone Y and per-point back-substitution stay on
    grouped = {int(p) for g_ in range(blk.shape[0]) for p in blk[g_, HDR_PT:HDR_PT + blk[g_, 1]]}
    assert len(grouped) == sum(int(blk[g_, 1]) for g_ in range(blk.shape[0]))
    # the two ineligible landmarks are lone points (in the lone range), not grouped
    assert len(grouped) == int(info[4] - info[3]) - 2
    assert max(int(pes[p + 1] - pes[p]) for p in range(int(info[3]), int(info[4]))) == 11
