"""Synthetic generator: deterministic, structure as SURVEY.md §8(d)."""
import numpy as np

from dynosam_amd import synth


def test_deterministic():
    g1, v1, t1 = synth.generate("T2")
    g2, v2, t2 = synth.generate("T2")
    assert np.array_equal(v1.data, v2.data) and np.array_equal(v1.keys, v2.keys)
    for t in g1.arrays():
        for a, b in zip(g1.arrays()[t], g2.arrays()[t]):
            if a is not None:
                assert np.array_equal(a, b)
    g3, v3, _ = synth.generate("T2", seed=43)
    assert not np.array_equal(v1.data, v3.data)


def test_counts_follow_formulation():
    F, O, S, P, Ls, Ld = 20, 2, 120, 4, 8, 10
    g, v, _ = synth.generate("T2")
    assert g.count("prior") == 1
    # odometry F-1 plus smoothing Betweens
    assert g.count("between") >= F - 1
    n_static_factors = S * (Ls - 1)
    n_dyn_points = int((v.kinds == 1).sum()) - S
    assert g.count("pose_to_point") == n_static_factors + n_dyn_points
    # each tracklet: Ld-1 points, Ld-2 ternaries
    assert g.count("landmark_motion_ternary") * (Ld - 1) == n_dyn_points * (Ld - 2)


def test_llworld_variant():
    g, v, _ = synth.generate("T2", formulation=1)
    assert g.count("landmark_motion_ternary") == 0
    assert g.count("landmark_motion_pose") > 0
    assert g.count("landmark_pose_smoothing") > 0
