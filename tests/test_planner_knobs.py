"""The planner's A/B knobs (INTEGRATION.md "Environment knobs") keep the plan
valid. Each knob is read once per process, so every setting runs in a
subprocess of its own (host-only planning, no GPU):
  * DYNOHIP_QCOST, DYNOHIP_QUEUE_ORDER=level, DYNOHIP_PLAN_SPIN_US=0,
    DYNOHIP_PLAN_WORKERS=1: the same tasks, dependencies and backward parts
    as the default plan, the dataflow queue still a topological order;
  * DYNOHIP_UPD_GROUP=3: update tasks regrouped, every contribution pair
    still applied exactly once, queue topological;
  * DYNOHIP_BACK_PART_TILES=2: every backward task split into parts of at
    most two entries that cover its entries in order;
  * DYNOHIP_PART_BALANCE=0: the partitioned plans' queues topological;
  * DYNOHIP_PLAN_TIMING, DYNOHIP_SCHED_TIMING: stage times on stderr, same plan."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_SCRIPT = r"""
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from dynosam_amd import synth
from dynosam_amd.optimizer import plan_export
name, nranks = sys.argv[2], int(sys.argv[3])
g, v, _ = synth.generate(name)
out = {}
for rank in range(nranks):
    pre = f"r{rank}_"
    for k in ("ftask", "fdep_start", "fdep", "fqueue", "pairs", "bpart", "bent", "flevel"):
        out[pre + k] = np.asarray(plan_export(g, v, k, nranks=nranks, rank=rank)).ravel().tolist()
print(json.dumps(out))
"""


def plan_with(env, name="C1", nranks=1):
    e = dict(os.environ)
    e.update(env)
    r = subprocess.run([sys.executable, "-c", _SCRIPT, ROOT, name, str(nranks)], capture_output=True, text=True,
                       env=e, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return {k: np.asarray(v, dtype=np.int64) for k, v in json.loads(r.stdout.strip().splitlines()[-1]).items()}


def topological(p, pre="r0_"):
    ft = p[pre + "ftask"].reshape(-1, 10)
    fs, fd, qu = p[pre + "fdep_start"], p[pre + "fdep"].reshape(-1, 2), p[pre + "fqueue"]
    n = ft.shape[0]
    assert sorted(qu.tolist()) == list(range(n))
    pos = np.empty(n, dtype=np.int64)
    pos[qu] = np.arange(n)
    writer, cnt = {}, {}
    for q in range(n):
        if ft[q, 0] == 1 or ft[q, 1] != ft[q, 2]:
            c = cnt.get(int(ft[q, 3]), 0) + 1
            cnt[int(ft[q, 3])] = c
            writer[(int(ft[q, 3]), c)] = q
    for q in range(n):
        for j in range(fs[q], fs[q + 1]):
            assert pos[writer[(int(fd[j, 0]), int(fd[j, 1]))]] < pos[q]


def pair_multiset(p, pre="r0_"):
    """(target slot, operand a, operand b) of every pair an update task or a
    panel applies (TileTask: kind, k, i, dst, diag, pd_beg, pd_end, po_beg,
    po_end, ...; a panel's pd pairs update its diagonal tile)"""
    ft = p[pre + "ftask"].reshape(-1, 10)
    pr = p[pre + "pairs"].reshape(-1, 2)
    out = []
    for t in ft:
        kind, dst, diag, pdb, pde, pob, poe = t[0], t[3], t[4], t[5], t[6], t[7], t[8]
        for e in range(pob, poe):
            out.append((int(dst), int(pr[e, 0]), int(pr[e, 1])))
        if kind == 0 and t[1] == t[2]:
            for e in range(pdb, pde):
                out.append((int(diag), int(pr[e, 0]), int(pr[e, 1])))
    return sorted(out)


@pytest.fixture(scope="module")
def base():
    return plan_with({})


@pytest.mark.parametrize("env", [{"DYNOHIP_QCOST": "12,9,2,4"}, {"DYNOHIP_QUEUE_ORDER": "level"},
                                 {"DYNOHIP_PLAN_SPIN_US": "0"}, {"DYNOHIP_PLAN_WORKERS": "1"}])
def test_order_knobs_keep_the_tasks(base, env):
    p = plan_with(env)
    for k in ("r0_ftask", "r0_fdep_start", "r0_fdep", "r0_pairs", "r0_bpart", "r0_bent", "r0_flevel"):
        assert np.array_equal(p[k], base[k]), (env, k)
    topological(p)
    if "DYNOHIP_QUEUE_ORDER" in env:
        assert np.array_equal(p["r0_fqueue"], np.arange(p["r0_ftask"].size // 10))


def test_update_grouping_applies_every_pair_once(base):
    p = plan_with({"DYNOHIP_UPD_GROUP": "3"})
    topological(p)
    assert pair_multiset(p) == pair_multiset(base)
    assert p["r0_ftask"].size <= base["r0_ftask"].size


def test_backward_parts_of_two_tiles(base):
    p = plan_with({"DYNOHIP_BACK_PART_TILES": "2"})
    bp = p["r0_bpart"].reshape(-1, 8)   # k, beg, end, nparts, part, pbase, pad, pad
    assert np.array_equal(p["r0_bent"], base["r0_bent"])
    assert (bp[:, 2] - bp[:, 1] <= 2).all() and (bp[:, 2] >= bp[:, 1]).all()
    i = 0
    while i < bp.shape[0]:
        n = bp[i, 3]
        parts = bp[i:i + n]
        assert (parts[:, 0] == parts[0, 0]).all() and list(parts[:, 4]) == list(range(n))
        assert (parts[1:, 1] == parts[:-1, 2]).all()   # contiguous, in order
        i += n


def test_midpoint_partition_queues_are_topological():
    p = plan_with({"DYNOHIP_PART_BALANCE": "0"}, name="C1", nranks=2)
    for rank in range(2):
        topological(p, f"r{rank}_")


def test_timing_knobs_print_and_keep_the_plan(base):
    """DYNOHIP_PLAN_TIMING / DYNOHIP_SCHED_TIMING only add per-stage times on
    stderr: the plan is the default one."""
    e = dict(os.environ, DYNOHIP_PLAN_TIMING="1", DYNOHIP_SCHED_TIMING="1")
    r = subprocess.run([sys.executable, "-c", _SCRIPT, ROOT, "C1", "1"], capture_output=True, text=True, env=e,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "[plan]" in r.stderr and "[tiles]" in r.stderr, r.stderr[-2000:]
    p = {k: np.asarray(v, dtype=np.int64) for k, v in json.loads(r.stdout.strip().splitlines()[-1]).items()}
    for k in base:
        assert np.array_equal(p[k], base[k]), k
