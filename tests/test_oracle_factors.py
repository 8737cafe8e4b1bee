"""Oracle factor / SE(3) restatement checks (CPU).

Pins: the reference's own known-answer tests for the hot-path factors
(dynosam/test/test_factors.cc:143-203: LandmarkMotionTernaryFactor analytic
Jacobians == gtsam::numericalDerivative3x at assert_equal's default 1e-9,
and zero residual at the exact motion), restated with the committed
Sampler(seed 42) draw in tests/golden/ternary_perturbation.json.
"""
import json
import os

import numpy as np
import pytest

import oracle_binding as ob

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "ternary_perturbation.json")))
SLOTS = {0: (0, 1), 1: (1, 1, 0), 2: (0, 0), 3: (0,), 4: (1, 1, 0, 0), 5: (0, 0, 0)}


def pose(w, t):
    T = ob.pose_expmap(np.concatenate([w, [0, 0, 0]]))
    T[9:12] = t
    return T


def retract(kind, x, d):
    if kind == 0:
        return ob.pose_compose(x, ob.pose_expmap(d))
    return x + d


def numerical_jacobian(ftype, vars_list, meas=None, delta=1e-5):
    """gtsam::numericalDerivative11 per slot (central, Local = difference)."""
    r0, _ = ob.eval_factor(ftype, np.concatenate(vars_list), meas)
    cols = []
    for s, kind in enumerate(SLOTS[ftype]):
        dim = 6 if kind == 0 else 3
        for j in range(dim):
            dx = np.zeros(dim)
            dx[j] = delta
            vp = list(vars_list)
            vp[s] = retract(kind, vars_list[s], dx)
            y1, _ = ob.eval_factor(ftype, np.concatenate(vp), meas)
            vp[s] = retract(kind, vars_list[s], -dx)
            y2, _ = ob.eval_factor(ftype, np.concatenate(vp), meas)
            cols.append(((y1 - r0) - (y2 - r0)) * (1.0 / (2.0 * delta)))
    return np.stack(cols, axis=1)


def golden_inputs():
    H = pose(GOLD["H_rodrigues"], GOLD["H_t"])
    Hp = ob.pose_compose(H, ob.pose_expmap(np.array(GOLD["perturb_tangent"])))  # Retract(H, delta)
    P1 = np.array(GOLD["P1"])
    P2 = ob.pose_compose(H, np.concatenate([np.eye(3).ravel(), P1]))[9:12]  # H * P1
    return H, Hp, P1, P2


def test_ternary_jacobians_match_numerical():
    # test_factors.cc:143-183
    H, Hp, P1, P2 = golden_inputs()
    r, J = ob.eval_factor(1, np.concatenate([P1, P2, Hp]))
    Jn = numerical_jacobian(1, [P1, P2, Hp])
    np.testing.assert_allclose(J, Jn, atol=1e-9, rtol=0)


def test_ternary_zero_error():
    # test_factors.cc:185-203
    H, Hp, P1, P2 = golden_inputs()
    r, _ = ob.eval_factor(1, np.concatenate([P1, P2, H]))
    assert np.max(np.abs(r)) < 1e-4
    assert np.max(np.abs(r)) < 1e-12


@pytest.mark.parametrize("seed", range(5))
def test_pose_to_point_jacobians(seed):
    rng = np.random.default_rng(seed)
    T = pose(rng.normal(0, 0.5, 3), rng.normal(0, 2, 3))
    p = rng.normal(0, 5, 3)
    z = rng.normal(0, 1, 3)
    r, J = ob.eval_factor(0, np.concatenate([T, p]), z)
    np.testing.assert_allclose(J, numerical_jacobian(0, [T, p], z), atol=1e-8)


@pytest.mark.parametrize("seed", range(5))
def test_between_fast_jacobians_exact_at_zero_residual(seed):
    # GTSAM BetweenFactor without GTSAM_SLOW_BUT_CORRECT_BETWEENFACTOR:
    # H1 = -Ad(hx^-1), H2 = I -- the true derivative when Local(z, hx) = 0
    rng = np.random.default_rng(seed)
    a = pose(rng.normal(0, 0.5, 3), rng.normal(0, 2, 3))
    b = pose(rng.normal(0, 0.5, 3), rng.normal(0, 2, 3))
    z = ob.pose_compose(ob.pose_inverse(a), b)
    r, J = ob.eval_factor(2, np.concatenate([a, b]), z)
    assert np.max(np.abs(r)) < 1e-12
    np.testing.assert_allclose(J, numerical_jacobian(2, [a, b], z), atol=1e-7)
    # away from zero residual the Jacobian is still the fast one (not the numeric)
    z2 = ob.pose_compose(z, ob.pose_expmap(rng.normal(0, 0.2, 6)))
    r2, J2 = ob.eval_factor(2, np.concatenate([a, b]), z2)
    np.testing.assert_allclose(J2, J, atol=1e-12)


def test_prior_identity_jacobian():
    rng = np.random.default_rng(3)
    x = pose(rng.normal(0, 0.5, 3), rng.normal(0, 2, 3))
    z = ob.pose_compose(x, ob.pose_expmap(rng.normal(0, 0.1, 6)))
    r, J = ob.eval_factor(3, x, z)
    np.testing.assert_allclose(J, np.eye(6), atol=0)
    # r = -Logmap(x^-1 z) = Logmap(z^-1 x)
    np.testing.assert_allclose(r, ob.pose_logmap(ob.pose_compose(ob.pose_inverse(z), x)), atol=1e-12)


@pytest.mark.parametrize("ftype", [4, 5])
def test_llworld_numerical_factors(ftype):
    # LandmarkMotionPose / LandmarkPoseSmoothing use numericalDerivative4x/3x
    rng = np.random.default_rng(ftype)
    if ftype == 4:
        vars_list = [rng.normal(0, 3, 3), rng.normal(0, 3, 3),
                     pose(rng.normal(0, 0.3, 3), rng.normal(0, 2, 3)), pose(rng.normal(0, 0.3, 3), rng.normal(0, 2, 3))]
    else:
        vars_list = [pose(rng.normal(0, 0.3, 3), rng.normal(0, 2, 3)) for _ in range(3)]
    r, J = ob.eval_factor(ftype, np.concatenate(vars_list))
    np.testing.assert_allclose(J, numerical_jacobian(ftype, vars_list), atol=1e-12)


def test_motion_pose_residual_formula():
    # LandmarkMotionPoseFactor.cc:83-88
    rng = np.random.default_rng(11)
    mp, mc = rng.normal(0, 3, 3), rng.normal(0, 3, 3)
    Lp, Lc = pose(rng.normal(0, 0.3, 3), rng.normal(0, 2, 3)), pose(rng.normal(0, 0.3, 3), rng.normal(0, 2, 3))
    r, _ = ob.eval_factor(4, np.concatenate([mp, mc, Lp, Lc]))
    C = ob.pose_compose(Lc, ob.pose_inverse(Lp))
    q = C[:9].reshape(3, 3) @ mp + C[9:]
    np.testing.assert_allclose(r, mc - q, atol=1e-12)


@pytest.mark.parametrize("theta", [0.0, 1e-9, 1e-4, 0.5, 2.0, 3.0, np.pi - 1e-4, np.pi - 1e-7])
def test_se3_exp_log_roundtrip(theta):
    rng = np.random.default_rng(int(theta * 1000))
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    xi = np.concatenate([axis * theta, rng.normal(0, 1, 3)])
    T = ob.pose_expmap(xi)
    R = T[:9].reshape(3, 3)
    np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-12)
    xi2 = ob.pose_logmap(T)
    tol = 1e-6 if theta > np.pi - 1e-3 else 1e-9
    np.testing.assert_allclose(xi2, xi, atol=tol)
