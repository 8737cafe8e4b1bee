"""Graph-file format (dynosam_amd/graphio.py, mirroring
FactorGraphTools.cc:256-381) and the testCliques fixture
(test_rgbd_backend.cc:272-486) checked on the CPU oracle."""
import json
import os

import numpy as np
import pytest

from dynosam_amd import _abi, graphio, synth
from dynosam_amd.keys import camera_pose_key, dynamic_landmark_key, object_motion_key, static_landmark_key
from oracle_binding import Oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def values_by_key(values, data=None):
    data = values.data if data is None else data
    off = values._offsets()
    return {int(k): np.asarray(data[off[i]:off[i + 1]]) for i, k in enumerate(values.keys)}


def assert_graphs_equal(g1, g2, pose_tol=1e-14):
    a1, a2 = g1.arrays(), g2.arrays()
    for t in _abi.FACTOR_TYPES:
        k1, m1, s1, h1 = a1[t]
        k2, m2, s2, h2 = a2[t]
        assert np.array_equal(k1, k2), t
        np.testing.assert_allclose(s1, s2, rtol=1e-15)
        assert np.array_equal(h1, h2), t
        if m1 is not None:
            np.testing.assert_allclose(m1, m2, rtol=0, atol=pose_tol * max(1.0, np.abs(m1).max(initial=0)))


@pytest.mark.parametrize("kw", [{}, {"formulation": 1}, {"robust": 0}])
def test_round_trip_synthetic(tmp_path, kw):
    g, v, _ = synth.generate("T2", **kw)
    p = tmp_path / "t2.graph"
    graphio.write(str(p), g, v)
    g2, v2 = graphio.read(str(p))
    assert_graphs_equal(g, g2)
    d1, d2 = values_by_key(v), values_by_key(v2)
    assert d1.keys() == d2.keys()
    for k in d1:
        np.testing.assert_allclose(d2[k], d1[k], rtol=0, atol=1e-14 * max(1.0, np.abs(d1[k]).max()))
    # a second round trip does not drift
    q = tmp_path / "t2b.graph"
    graphio.write(str(q), g2, v2)
    g3, _ = graphio.read(str(q))
    assert_graphs_equal(g2, g3)


def test_reference_precision_lines():
    # lines as the reference writes them (default 6 significant digits,
    # FactorGraphTools.hpp:414-438)
    X0, l0 = camera_pose_key(0), static_landmark_key(0)
    lines = [
        f"SE3_PRIOR_FACTOR {X0} 1 3 4 0.0997319 0.0498659 0.0598391 0.991961 100 0 0 0 0 0 100 0 0 0 0 100 0 0 0 100 0 0 100 0 100",
        f"SE3_POSE_VALUE {X0} 1 3 4 0.0997319 0.0498659 0.0598391 0.991961",
        f"POSE_TO_POINT_FACTOR {X0} {l0} 1 2 3 0.01 0 0 0.01 0 0.01",
        f"POINT3_STATIC_VALUE {l0} 0 1 1",
    ]
    g, v = graphio.read(lines)
    assert g.count("prior") == 1 and g.count("pose_to_point") == 1
    np.testing.assert_allclose(g.arrays()["prior"][2], [[0.1] * 6])
    np.testing.assert_allclose(g.arrays()["pose_to_point"][2], [[10.0] * 3])
    R = g.arrays()["prior"][1][0][:9].reshape(3, 3)
    np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-12)
    assert len(v) == 2


def test_rejections():
    X0, l0 = camera_pose_key(0), static_landmark_key(0)
    with pytest.raises(graphio.GraphFileError, match="diagonal"):
        graphio.read([f"POSE_TO_POINT_FACTOR {X0} {l0} 1 2 3 1 0.5 0 1 0 1"])
    with pytest.raises(graphio.GraphFileError, match="unknown tag"):
        graphio.read(["VERTEX_SE3:QUAT 0 0 0 0 0 0 0 1"])
    with pytest.raises(graphio.GraphFileError, match="information entries"):
        graphio.read([f"POSE_TO_POINT_FACTOR {X0} {l0} 1 2 3 1 0 0 1"])
    with pytest.raises(graphio.GraphFileError, match="twice"):
        graphio.read([f"POINT3_STATIC_VALUE {l0} 0 1 1", f"POINT3_STATIC_VALUE {l0} 0 1 1"])


def test_quaternion_round_trip():
    rng = np.random.default_rng(1)
    for _ in range(200):
        q = rng.standard_normal(4)
        q /= np.linalg.norm(q)
        R = graphio.quat_to_rot(*q)
        q2 = graphio.rot_to_quat(R)
        np.testing.assert_allclose(graphio.quat_to_rot(*q2), R, atol=1e-14)
    for R in (np.diag([1.0, -1, -1]), np.diag([-1.0, 1, -1]), np.diag([-1.0, -1, 1])):  # 180 degree turns
        np.testing.assert_allclose(graphio.quat_to_rot(*graphio.rot_to_quat(R)), R, atol=1e-14)


def cliques():
    return graphio.read(os.path.join(GOLDEN, "cliques.graph"))


def test_cliques_fixture_structure():
    g, v = cliques()
    assert g.count("pose_to_point") == 12 and g.count("landmark_motion_ternary") == 6
    assert g.count("between") == 2 and g.count("prior") == 1
    keys = set(int(k) for k in v.keys)
    assert keys == ({camera_pose_key(k) for k in range(3)} | {static_landmark_key(0)} |
                    {dynamic_landmark_key(k, t) for k in range(3) for t in (1, 2, 3)} |
                    {object_motion_key(1, 1), object_motion_key(1, 2)})
    # H_{1,1}, H_{1,2} start at identity (test_rgbd_backend.cc:472-473)
    d = values_by_key(v)
    np.testing.assert_array_equal(d[object_motion_key(1, 1)], np.r_[np.eye(3).ravel(), 0, 0, 0])


def test_oracle_reproduces_cliques_golden():
    gold = json.load(open(os.path.join(GOLDEN, "lm_cliques.json")))
    g, v = cliques()
    o = Oracle(g, v)
    s = o.optimize()
    assert (s.iterations, s.inner_iterations) == (gold["iterations"], gold["inner_iterations"])
    assert s.final_error == pytest.approx(gold["final_error"], rel=1e-12)
    tr = o.trace()
    assert len(tr) == len(gold["trace"])
    for a, b in zip(tr, gold["trace"]):
        for f in ("lam", "accepted", "solved", "stop"):
            assert a[f] == b[f]
        assert a["new_error"] == pytest.approx(b["new_error"], rel=1e-12)
    out = values_by_key(v, o.values_data())
    for k, ref in gold["final_values"].items():
        np.testing.assert_allclose(out[int(k)], ref, rtol=0, atol=1e-12 * max(1.0, np.abs(ref).max()))
