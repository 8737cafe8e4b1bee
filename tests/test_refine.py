"""Batched object-motion refinement:
dynosam_amd/csrc/refine.hip through dynosam_amd.refine vs the numpy
restatement oracle/refine.py of MotionOnlyRefinementOptimizer::optimize
(MotionSolver-inl.hpp:277-470).

The reference has no test for this optimiser, so its outputs are "parity
unpinned" against GTSAM itself; the restatement's factors are pinned by
analytic-vs-numerical Jacobian checks, and the GPU must reproduce the
restatement: the same LM iteration / inner-iteration counts, status and
outlier sets, and the motion within 1e-6 relative Frobenius.
"""
import os
import sys

import numpy as np
import pytest

from dynosam_amd import refine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import refine as orf  # noqa: E402  (test infrastructure: the checker)


def _num_jac(f, x, retract, dim, h=1e-6):
    cols = []
    for j in range(dim):
        e = np.zeros(dim)
        e[j] = h
        cols.append((f(retract(x, e)) - f(retract(x, -e))) / (2 * h))
    return np.stack(cols, axis=1)


def test_projection_jacobians_match_numerical():
    rng = np.random.default_rng(0)
    for _ in range(10):
        T = orf.pose_expmap(rng.normal(0, 0.5, 6))
        p = T[1] + T[0] @ np.array([rng.normal(0, 1), rng.normal(0, 1), 6.0 + rng.normal(0, 1)])
        K = np.array([480.0, 520.0, 0.7, 320.0, 240.0])
        kp = np.array([310.0, 250.0])
        r, Jx, Jp = orf.project(T, p, K, kp)
        Nx = _num_jac(lambda X: orf.project(X, p, K, kp)[0], T, orf.retract, 6)
        Np = _num_jac(lambda q: orf.project(T, q, K, kp)[0], p, lambda a, e: a + e, 3)
        np.testing.assert_allclose(Jx, Nx, rtol=0, atol=1e-6 * np.abs(Jx).max())
        np.testing.assert_allclose(Jp, Np, rtol=0, atol=1e-6 * np.abs(Jp).max())


def test_projection_cheirality():
    T = (np.eye(3), np.zeros(3))
    r, Jx, Jp = orf.project(T, np.array([0.0, 0.0, -1.0]), np.array([500.0, 500, 0, 320, 240]), np.zeros(2))
    assert np.all(r == 1000.0) and not Jx.any() and not Jp.any()


def test_ternary_jacobians_match_numerical():
    rng = np.random.default_rng(1)
    H = orf.pose_expmap(rng.normal(0, 0.5, 6))
    p1, p2 = rng.normal(0, 2, 3), rng.normal(0, 2, 3)
    r, J1, J2, J3 = orf.ternary(p1, p2, H)
    add = lambda a, e: a + e  # noqa: E731
    np.testing.assert_allclose(J1, _num_jac(lambda q: orf.ternary(q, p2, H)[0], p1, add, 3), atol=1e-8)
    np.testing.assert_allclose(J2, _num_jac(lambda q: orf.ternary(p1, q, H)[0], p2, add, 3), atol=1e-8)
    np.testing.assert_allclose(J3, _num_jac(lambda X: orf.ternary(p1, p2, X)[0], H, orf.retract, 6), atol=1e-7)


def test_oracle_chi2_threshold():
    from scipy.stats import chi2
    assert orf.CHI2_3_099 == pytest.approx(chi2.ppf(0.99, 3), rel=1e-12)


def test_params_default():
    import ctypes as C
    from dynosam_amd import _abi, _native
    p = _abi.RefineParams()
    _native.load("libdynohip.so").dynorefine_params_default(C.byref(p))
    assert (p.landmark_motion_sigma, p.projection_sigma, p.k_huber, p.prior_sigma, p.outlier_reject) == \
        (0.001, 2.0, 0.0001, 1e-5, 1)


# ------------------------------------------------------------------ GPU ----
def _oracle_run(batch, params):
    R = orf.Refiner(schur=True, **params)
    out = []
    for p in range(batch.n):
        d = batch.problem(p)
        pb = orf.Problem(d["X_k_1"], d["X_k"], d["H"], d["K"], d["kp_k_1"], d["kp_k"], d["m_k_1"], d["m_k"])
        out.append(R.refine(pb))
    return out


def _shift_every_fifth(batch):
    kp = batch.kp_k.copy()
    for p in range(batch.n):
        a, b = batch.track_start[p], batch.track_start[p + 1]
        kp[a:b:5] += 25.0
    return kp


def _compare(batch, H, flags, res, ref):
    """Free-running: integer outcomes (status, outlier sets) identical, the
    motion within 1e-3. Huber k = 1e-4 puts every factor in its linear (L1)
    regime and the priors (sigma 1e-5) make the system condition number
    ~1e15, so the LM walks a flat valley: trajectories that agree per step
    stop a few iterations apart near the relativeErrorTol threshold, at
    points of the valley up to ~1e-4 apart. The north-star per-iteration bar
    (1e-6) is checked conditioned (test_refine_per_iteration_conditioned)."""
    for p, r in enumerate(ref):
        got = res[p]
        assert got["status"] == r["status"], p
        assert abs(got["iterations"] - r["iterations"]) <= 4, (p, got, r["iterations"])
        Href = orf.p12(r["state"][2])
        assert np.linalg.norm(H[p] - Href) / np.linalg.norm(Href) < 1e-3, p
        assert got["error_before"] == pytest.approx(r["error_before"], rel=1e-9)
        # both stop in the flat valley: decreased, and within 20% of each other
        assert got["error_after"] <= got["error_before"] and r["error_after"] <= r["error_before"]
        assert got["error_after"] == pytest.approx(r["error_after"], rel=0.2, abs=1e-12)
        a = batch.track_start[p]
        assert sorted(np.nonzero(flags[a:batch.track_start[p + 1]])[0].tolist()) == sorted(r["outliers"]), p
        assert got["n_outliers"] == len(r["outliers"])


@pytest.mark.gpu
@pytest.mark.parametrize("params", [{}, dict(landmark_motion_sigma=0.01, projection_sigma=0.5)])
def test_refine_per_iteration_conditioned(gpu_available, params):
    """Per LM iteration, from the oracle's state and lambda: one GPU
    iterate() must land on the oracle's next state (motion within 1e-6
    relative Frobenius, the north-star bar) with the same error."""
    from dynosam_amd import _abi
    batch = refine.synthetic_batch(6, tracks=(5, 90), seed=21, behind_camera=1)
    if params:
        batch.kp_k = _shift_every_fifth(batch)
    R = orf.Refiner(outlier_reject=0, schur=True, **params)
    cases = []  # (problem, state_i, lambda_i, state_i+1)
    for p in range(batch.n):
        d = batch.problem(p)
        pb = orf.Problem(d["X_k_1"], d["X_k"], d["H"], d["K"], d["kp_k_1"], d["kp_k"], d["m_k_1"], d["m_k"])
        hist = R.optimize(pb)["history"]
        for i in range(len(hist) - 1):
            cases.append((p, hist[i][0], hist[i][1], hist[i + 1][0]))
    assert len(cases) > 40
    opt = refine.MotionOnlyRefinementOptimizer(outlier_reject=0, **params)
    for lam in sorted({c[2] for c in cases}):
        sel = [c for c in cases if c[2] == lam]
        counts = [batch.track_start[c[0] + 1] - batch.track_start[c[0]] for c in sel]
        ts = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
        b = refine.RefineBatch(
            ts, np.stack([batch.X_k_1[c[0]] for c in sel]), np.stack([batch.X_k[c[0]] for c in sel]),
            np.stack([orf.p12(c[1][2]) for c in sel]), np.stack([batch.calibration[c[0]] for c in sel]),
            np.concatenate([batch.problem(c[0])["kp_k_1"] for c in sel]),
            np.concatenate([batch.problem(c[0])["kp_k"] for c in sel]),
            np.concatenate([c[1][3] for c in sel]), np.concatenate([c[1][4] for c in sel]),
            X_k_1_init=np.stack([orf.p12(c[1][0]) for c in sel]), X_k_init=np.stack([orf.p12(c[1][1]) for c in sel]))
        lm = _abi.LMParams.gtsam_default()
        lm.lambda_initial = lam
        lm.max_iterations = 1
        H, _, res = opt.optimize_batch(b, lm)
        for j, c in enumerate(sel):
            Href = orf.p12(c[3][2])
            assert np.linalg.norm(H[j] - Href) / np.linalg.norm(Href) < 1e-6, (c[0], lam)
            d = batch.problem(c[0])
            pb = orf.Problem(d["X_k_1"], d["X_k"], d["H"], d["K"], d["kp_k_1"], d["kp_k"], d["m_k_1"], d["m_k"])
            e_next = R.error(pb, *c[3])
            # the error also depends on the point depths along the viewing rays,
            # the system's near-null directions (condition ~1e17 at small lambda):
            # they follow the step only to ~1e-5
            assert res[j]["error_after"] == pytest.approx(e_next, rel=1e-4, abs=1e-14), (c[0], lam)


def _one_iteration_cases(batch, hist_of):
    """(problem, state_i, lambda_i, state_i+1, inactive mask) for every LM
    iteration of hist_of(p)"""
    cases = []
    for p in range(batch.n):
        got = hist_of(p)
        if got is None:
            continue
        hist, inactive = got
        for i in range(len(hist) - 1):
            cases.append((p, hist[i][0], hist[i][1], hist[i + 1][0], inactive, i))
    return cases


def _gpu_one_iteration(batch, opt, sel):
    """One GPU LM iteration (max_iterations 1) from each case's state and
    lambda, grouped by lambda; returns H per case"""
    from dynosam_amd import _abi
    counts = [batch.track_start[c[0] + 1] - batch.track_start[c[0]] for c in sel]
    ts = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    b = refine.RefineBatch(
        ts, np.stack([batch.X_k_1[c[0]] for c in sel]), np.stack([batch.X_k[c[0]] for c in sel]),
        np.stack([orf.p12(c[1][2]) for c in sel]), np.stack([batch.calibration[c[0]] for c in sel]),
        np.concatenate([batch.problem(c[0])["kp_k_1"] for c in sel]),
        np.concatenate([batch.problem(c[0])["kp_k"] for c in sel]),
        np.concatenate([c[1][3] for c in sel]), np.concatenate([c[1][4] for c in sel]),
        X_k_1_init=np.stack([orf.p12(c[1][0]) for c in sel]), X_k_init=np.stack([orf.p12(c[1][1]) for c in sel]),
        ternary_inactive=np.concatenate([c[4] for c in sel]))
    lm = _abi.LMParams.gtsam_default()
    lm.lambda_initial = sel[0][2]
    lm.max_iterations = 1
    H, _, res = opt.optimize_batch(b, lm)
    return H, res


def _max_point_block_cond(R, pb, state, lam):
    """Largest condition number of the damped 3x3 point blocks J_p^T J_p + lam I
    of the tracklets whose ternary factor is out of the graph (their points
    keep only one projection each: the depth along the ray is unobserved)"""
    blocks = {}
    for f in R.factors(pb, *state):
        if f[0] != "proj":
            continue
        for v, J in f[2].items():
            if v >= 3 and not pb.active[(v - 3) // 2]:
                blocks[v] = blocks.get(v, np.zeros((3, 3))) + J.T @ J
    worst = 0.0
    for M in blocks.values():
        ev = np.linalg.eigvalsh(M + lam * np.eye(3))
        worst = max(worst, np.inf if ev[0] <= 0 else ev[-1] / ev[0])
    return worst


@pytest.mark.gpu
def test_refine_mode2_resolve_per_iteration_conditioned(gpu_available):
    """outlier_reject = 2: the re-solve after the outlier ternaries are
    dropped (MotionSolver-inl.hpp:405-437, the loop the code intends),
    conditioned per LM iteration: from the oracle's state, lambda and active
    set, one GPU iteration against the oracle's next state.

    Root cause of the round-1 free-running divergence: a tracklet whose
    ternary is dropped keeps one projection per point, so each point's depth
    along its ray is unobserved; near convergence the projections sit inside
    the Huber threshold (full weight), J_p^T J_p reaches ~1e11 and the damped
    3x3 block's condition number (1e11 / lambda) passes 1/eps once lambda
    <= ~1e-5. Whether that block's Cholesky succeeds is then decided by
    rounding, so the GPU and the oracle can take different accept / reject
    paths from the same state (a failed solve raises lambda, as GTSAM's
    IndeterminantLinearSystemException does). The check: wherever both take
    the same inner tries, the motion agrees within the north-star 1e-6;
    wherever they differ, the oracle confirms a numerically singular point
    block (condition > 1e15) at that state and lambda."""
    batch = refine.synthetic_batch(12, tracks=(10, 40), seed=5, outlier_frac=0.15)
    batch.kp_k = _shift_every_fifth(batch)
    params = dict(landmark_motion_sigma=0.01, projection_sigma=0.5)
    R = orf.Refiner(outlier_reject=0, schur=True, **params)
    tries, pbs = {}, {}

    def second_round(p):
        d = batch.problem(p)
        pb = orf.Problem(d["X_k_1"], d["X_k"], d["H"], d["K"], d["kp_k_1"], d["kp_k"], d["m_k_1"], d["m_k"])
        r1 = R.optimize(pb)
        outl = R.outliers(pb, r1["state"])
        if not outl:
            return None
        pb.active[outl] = False
        st = r1["state"]
        pb.X1, pb.X2, pb.H = st[0], st[1], st[2]
        pb.P1, pb.P2 = st[3].copy(), st[4].copy()
        r2 = R.optimize(pb)
        # inner tries per outer iteration (a group of the trace ends at an accept)
        groups, cur = [], []
        for e in r2["trace"]:
            cur.append(e)
            if e["accepted"]:
                groups.append(len(cur))
                cur = []
        tries[p] = groups
        pbs[p] = pb
        return r2["history"], ~pb.active

    cases = _one_iteration_cases(batch, second_round)
    assert len(cases) > 10 and any(c[4].any() for c in cases)
    opt = refine.MotionOnlyRefinementOptimizer(outlier_reject=0, **params)
    same, diverged = [], []
    for lam in sorted({c[2] for c in cases}):
        sel = [c for c in cases if c[2] == lam]
        H, res = _gpu_one_iteration(batch, opt, sel)
        for j, c in enumerate(sel):
            p, it = c[0], c[5]
            if it >= len(tries[p]):
                continue
            dev = np.linalg.norm(H[j] - orf.p12(c[3][2])) / np.linalg.norm(orf.p12(c[3][2]))
            if res[j]["inner_iterations"] == tries[p][it]:
                same.append((p, it, lam, dev))
            else:
                diverged.append((p, it, lam, _max_point_block_cond(R, pbs[p], c[1], lam)))
    print(f"mode-2 re-solve: {len(same)} iterations on the same path, max motion dev "
          f"{max(d[3] for d in same):.1e}; {len(diverged)} diverged, min point-block condition "
          f"{min([d[3] for d in diverged] or [np.inf]):.1e}")
    assert len(same) >= len(diverged) and len(same) > 20
    for d in same:
        assert d[3] < 1e-6, d
    for d in diverged:
        assert d[3] > 1e15, d


@pytest.mark.gpu
def test_refine_batch_matches_oracle(gpu_available):
    # up to 150 tracks per problem: several 64-lane chunks; points behind the camera
    batch = refine.synthetic_batch(20, tracks=(3, 150), seed=11, behind_camera=2)
    opt = refine.MotionOnlyRefinementOptimizer()
    H, flags, res = opt.optimize_batch(batch)
    _compare(batch, H, flags, res, _oracle_run(batch, {}))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_refine_outlier_modes_match_oracle(gpu_available, mode):
    batch = refine.synthetic_batch(12, tracks=(10, 40), seed=5, outlier_frac=0.15)
    batch.kp_k = _shift_every_fifth(batch)
    params = dict(landmark_motion_sigma=0.01, projection_sigma=0.5, outlier_reject=mode)
    opt = refine.MotionOnlyRefinementOptimizer(**params)
    H, flags, res = opt.optimize_batch(batch)
    ref = _oracle_run(batch, params)
    if mode:
        assert any(r["outliers"] for r in ref)  # the case exercises the outlier step
    if mode < 2:
        _compare(batch, H, flags, res, ref)
        return
    # mode 2 (the loop the reference intends, a documented deviation): after the
    # outlier ternaries are dropped those points keep only their projections,
    # so their depths are undetermined up to lambda and the L1-like valley in H
    # is flatter still; the continuous result depends on the elimination
    # rounding. Integer outcomes must agree exactly.
    for p, r in enumerate(ref):
        assert res[p]["status"] == r["status"]
        a, b = batch.track_start[p], batch.track_start[p + 1]
        assert sorted(np.nonzero(flags[a:b])[0].tolist()) == sorted(r["outliers"]), p
        assert res[p]["error_after"] <= res[p]["error_before"]


@pytest.mark.gpu
def test_refine_bit_reproducible_and_empty(gpu_available):
    batch = refine.synthetic_batch(64, tracks=(0, 80), seed=2)
    opt = refine.MotionOnlyRefinementOptimizer()
    a = opt.optimize_batch(batch)
    opt.solve()
    b = opt.download()
    np.testing.assert_array_equal(a[0], b[0])
    assert a[2] == b[2]
    empty = [p for p in range(batch.n) if batch.track_start[p] == batch.track_start[p + 1]]
    for p in empty:  # priors only: nothing moves the motion
        np.testing.assert_array_equal(a[0][p], batch.H_init[p])
