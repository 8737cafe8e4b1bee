"""The host planner's parallel sections (csrc/plan.cpp: target-range gather
builds, per-worker counting sorts, chunked layout passes) reproduce the
single-threaded build bit for bit, and a plan rebuilt into recycled arrays
equals a fresh one: every plan field's digest
(dynohip_plan_export "digest") with the pool capped at one worker
(DYNOHIP_PLAN_WORKERS=1, in a child process: the pool is process-wide) equals
the digest with the default pool. Host only."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_plan_is_independent_of_planner_workers(tmp_path):
    path = str(tmp_path / "one_worker.npz")
    env = dict(os.environ, DYNOHIP_PLAN_WORKERS="1")
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "plan_digest.py"), "save", path], env=env,
                   check=True, timeout=600)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import plan_digest
    many = plan_digest.digests()
    one = np.load(path)
    assert sorted(many) == sorted(one.files)
    for k, x in many.items():
        y = one[k]
        assert x.shape == y.shape, k
        diff = np.nonzero((x.reshape(-1, 2) != y.reshape(-1, 2)).any(1))[0]
        assert diff.size == 0, "%s: fields %s differ" % (k, diff.tolist())


def test_recycled_plan_equals_fresh_plan():
    """build_plan into a Plan that held a plan already (plan_recycle keeps
    its arrays' capacity) gives the same plan as a fresh build."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import plan_digest
    fresh, again = plan_digest.digests(), plan_digest.digests("@recycled")
    for k, x in fresh.items():
        diff = np.nonzero((x.reshape(-1, 2) != again[k].reshape(-1, 2)).any(1))[0]
        assert diff.size == 0, "%s: fields %s differ" % (k, diff.tolist())


def test_small_plan_cap_equals_threaded_plan(tmp_path):
    """Graphs under the small-plan threshold (T2, C1, the LLWorld T2: values
    + factors < 20k) plan their parallel sections inline on the calling
    thread (plan.cpp small_plan_items). The same plans built with the cap
    off (DYNOHIP_SMALL_PLAN_ITEMS=0, the pool's threaded sections, in a
    child process) have identical digests, field by field."""
    path = str(tmp_path / "uncapped.npz")
    env = dict(os.environ, DYNOHIP_SMALL_PLAN_ITEMS="0", DYNOHIP_PLAN_WORKERS="4")
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "plan_digest.py"), "save", path], env=env,
                   check=True, timeout=600)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import plan_digest
    capped = plan_digest.digests()
    threaded = np.load(path)
    small = [k for k in capped if k.startswith(("T2", "C1"))]
    assert small, sorted(capped)
    for k in capped:
        diff = np.nonzero((capped[k].reshape(-1, 2) != threaded[k].reshape(-1, 2)).any(1))[0]
        assert diff.size == 0, "%s: fields %s differ" % (k, diff.tolist())


def test_value_key_index_errors_on_a_large_graph():
    """plan.cpp KeyIndex over a C2-sized value list (30k values):
    a duplicated value key or a bad value kind at the start, the middle or
    the end is reported (DYNOHIP_EINVAL), and the same graph without the
    defect plans."""
    from dynosam_amd import synth
    from dynosam_amd.graph import Values
    from dynosam_amd.optimizer import DynohipError, plan_export
    g, v, _ = synth.generate("C2")
    assert plan_export(g, v, "info")[0] > 0
    for where in (1, len(v) // 2, len(v) - 1):
        keys = v.keys.copy()
        keys[where] = keys[where - 1]   # a duplicate (the earlier copy keeps its index)
        try:
            plan_export(g, Values(keys, v.kinds, v.data), "info")
            raise AssertionError("duplicate value key accepted")
        except DynohipError as e:
            assert e.code == -1   # DYNOHIP_EINVAL
        kinds = v.kinds.copy()
        kinds[where] = 7
        try:
            plan_export(g, Values(v.keys, kinds, v.data), "info")
            raise AssertionError("bad value kind accepted")
        except DynohipError as e:
            assert e.code == -1
