"""TEST INFRASTRUCTURE — CPU restatement (numpy) of the frontend's object
motion refinement, MotionOnlyRefinementOptimizer::optimize with
RefinementSolver::ProjectionError
(dynosam/include/dynosam/frontend/vision/MotionSolver-inl.hpp:277-470), the
checker for the batched GPU solver (dynosam_amd/csrc/refine.hip). Only tests/
and bench.py's cpu_baseline leg may use it.

Per object and frame pair (k-1, k) the graph is
  PriorFactor<Pose3>(X_{k-1}), PriorFactor<Pose3>(X_k)     sigma 1e-5 (:307-309)
  per tracklet i, in order:
    GenericProjectionFactor<Pose3, Point3, Cal3_S2>(kp_{k-1}, X_{k-1}, m_{k-1})
    GenericProjectionFactor(kp_k, X_k, m_k)        Huber(k) on Isotropic(2, sigma_proj)
    LandmarkMotionTernaryFactor(m_{k-1}, m_k, H)   Huber(k) on Isotropic(3, sigma_motion)
with values X_{k-1}, X_k, H (initial motion) and the back-projected points,
solved by gtsam::LevenbergMarquardtOptimizer with default parameters (GTSAM
4.2 semantics as in oracle/oracle.c). Afterwards
factor_graph_tools::determineFactorOutliers<LandmarkMotionTernaryFactor>
(FactorGraphTools.hpp:70-98) flags ternary factors whose Gaussian error
exceeds 0.5 * chi2_quantile(3, 0.99).

GTSAM details restated here (GTSAM 4.2.0, not in /root/reference):
  * PinholeCamera<Cal3_S2>::project: q = X.transformTo(p); CheiralityException
    when q.z <= 0; pn = (q.x/q.z, q.y/q.z); uv = (fx pn.x + s pn.y + u0,
    fy pn.y + v0); Dpose = Dcal * [[u v, -(1+u^2), v, -d, 0, d u],
    [1+v^2, -u v, -u, 0, -d, d v]] with d = 1/q.z; Dpoint = Dcal * d *
    [[1, 0, -u], [0, 1, -v]] * R^T.
  * GenericProjectionFactor(throwCheirality=false): on CheiralityException
    the error is (2 fx, 2 fx) with zero Jacobians.
Outlier rejection: with outlier_reject (the default) and at least one outlier
the reference re-inserts the motion key into `values` (MotionSolver-inl.hpp:
416), which throws gtsam::ValuesKeyAlreadyExists; that outcome is reported as
status VALUES_KEY_EXISTS. outlier_reject = 2 runs the loop the code intends
(remove the outlier ternary factors, re-solve from the optimised values, at
most 4 times) — an explicit deviation, off by default.
"""
import numpy as np

CHI2_3_099 = 11.344866730144373  # boost chi_squared quantile(3, 0.99)
EPS = np.finfo(float).eps

OK, VALUES_KEY_EXISTS = 0, 1


def skew(w):
    return np.array([[0.0, -w[2], w[1]], [w[2], 0.0, -w[0]], [-w[1], w[0], 0.0]])


def rot_expmap(w):
    th2 = w @ w
    W = skew(w)
    if th2 <= EPS:
        return np.eye(3) + W
    th = np.sqrt(th2)
    K = W / th
    return np.eye(3) + np.sin(th) * K + 2.0 * np.sin(th / 2.0) ** 2 * (K @ K)


def rot_logmap(R):
    """gtsam::SO3::Logmap (GTSAM 4.2), as oracle/oracle.c restates it"""
    R11, R12, R13 = R[0]
    R21, R22, R23 = R[1]
    R31, R32, R33 = R[2]
    tr = R11 + R22 + R33
    if tr + 1.0 < 1e-3:
        if R33 > R22 and R33 > R11:
            W, Q1, Q2, Q3, order = R21 - R12, 2.0 + 2.0 * R33, R31 + R13, R23 + R32, (1, 2, 0)
        elif R22 > R11:
            W, Q1, Q2, Q3, order = R13 - R31, 2.0 + 2.0 * R22, R23 + R32, R12 + R21, (2, 0, 1)
        else:
            W, Q1, Q2, Q3, order = R32 - R23, 2.0 + 2.0 * R11, R12 + R21, R31 + R13, (0, 1, 2)
        r = np.sqrt(Q1)
        norm = np.sqrt(Q1 * Q1 + Q2 * Q2 + Q3 * Q3 + W * W)
        sgn_w = -1.0 if W < 0 else 1.0
        mag = np.pi - (2 * sgn_w * W) / norm
        scale = 0.5 * (1 / r) * mag
        Q = (Q1, Q2, Q3)
        return np.array([sgn_w * scale * Q[k] for k in order])
    tr_3 = tr - 3.0
    if tr_3 < -1e-6:
        theta = np.arccos((tr - 1.0) / 2.0)
        magnitude = theta / (2.0 * np.sin(theta))
    else:
        magnitude = 0.5 - tr_3 / 12.0 + tr_3 * tr_3 / 60.0
    return magnitude * np.array([R32 - R23, R13 - R31, R21 - R12])


def pose_expmap(xi):
    w, v = xi[:3], xi[3:]
    R = rot_expmap(w)
    th2 = w @ w
    if th2 > EPS:
        wxv = np.cross(w, v)
        t = (wxv - R @ wxv + w * (w @ v)) / th2
    else:
        t = v.copy()
    return R, t


def pose_logmap(R, t):
    w = rot_logmap(R)
    th = np.sqrt(w @ w)
    if th < 1e-10:
        return np.concatenate([w, t])
    Wn = skew(w / th)
    WT = Wn @ t
    u = t - (0.5 * th) * WT + (1.0 - th / (2.0 * np.tan(0.5 * th))) * (Wn @ WT)
    return np.concatenate([w, u])


def retract(T, xi):
    R, t = T
    dR, dt = pose_expmap(xi)
    return R @ dR, R @ dt + t


def p12(T):
    return np.concatenate([T[0].reshape(9), T[1]])


def T_of(a):
    a = np.asarray(a, float)
    return a[:9].reshape(3, 3).copy(), a[9:12].copy()


def huber_w(e, k):
    return 1.0 if e <= k else k / e


def huber_rho(e, k):
    return 0.5 * e * e if e <= k else k * (e - 0.5 * k)


class Problem:
    """One object/frame-pair refinement problem."""

    def __init__(self, X_k_1, X_k, H, K, kp_k_1, kp_k, m_k_1, m_k):
        self.X1, self.X2, self.H = T_of(X_k_1), T_of(X_k), T_of(H)
        self.prior1, self.prior2 = T_of(X_k_1), T_of(X_k)
        self.K = np.asarray(K, float)            # fx, fy, s, u0, v0
        self.kp1, self.kp2 = np.asarray(kp_k_1, float), np.asarray(kp_k, float)
        self.P1, self.P2 = np.asarray(m_k_1, float).copy(), np.asarray(m_k, float).copy()
        self.active = np.ones(len(self.P1), dtype=bool)  # ternary factors present


def project(T, p, K, kp):
    """GenericProjectionFactor::evaluateError: r (2), Dpose (2x6), Dpoint (2x3)"""
    R, t = T
    q = R.T @ (p - t)
    fx, fy, s, u0, v0 = K
    if q[2] <= 0:
        return np.array([2.0 * fx, 2.0 * fx]), np.zeros((2, 6)), np.zeros((2, 3))
    d = 1.0 / q[2]
    u, v = q[0] * d, q[1] * d
    r = np.array([fx * u + s * v + u0 - kp[0], fy * v + v0 - kp[1]])
    Dcal = np.array([[fx, s], [0.0, fy]])
    Dpn_pose = np.array([[u * v, -(1 + u * u), v, -d, 0.0, d * u], [1 + v * v, -u * v, -u, 0.0, -d, d * v]])
    Dpn_q = d * np.array([[1.0, 0.0, -u], [0.0, 1.0, -v]])
    return r, Dcal @ Dpn_pose, Dcal @ Dpn_q @ R.T


def ternary(p1, p2, H):
    """LandmarkMotionTernaryFactor.cc:37-73: r = m_{k-1} - H^-1 m_k"""
    R, t = H
    q = R.T @ (p2 - t)
    r = p1 - q
    J1 = np.eye(3)
    J2 = -R.T
    J3 = np.hstack([-skew(q), np.eye(3)])
    return r, J1, J2, J3


def prior(T, Z):
    """PriorFactor<Pose3>: r = -Local(x, prior), H = I"""
    R, t = T
    Ri = R.T
    e = (Ri @ Z[0], Ri @ (Z[1] - t))
    return -pose_logmap(*e)


class Refiner:
    def __init__(self, landmark_motion_sigma=0.001, projection_sigma=2.0, k_huber=0.0001, outlier_reject=1,
                 prior_sigma=1e-5, schur=False):
        """schur=False: dense Cholesky of the damped system (GTSAM's
        elimination is exact up to rounding; any order is equivalent in exact
        arithmetic). schur=True: eliminate every tracklet's 6x6 point block
        first, then the 18x18 pose system — the order the GPU kernel uses.
        The system's condition number reaches 1e15-1e17 (priors at sigma
        1e-5, Huber k 1e-4), so the two orders differ by up to ~1e-3 in the
        step at lambda ~1e-10; the per-iteration parity test pins the GPU to
        the same elimination order."""
        self.sm, self.sp, self.k, self.outlier_reject, self.sprior = (landmark_motion_sigma, projection_sigma,
                                                                      k_huber, outlier_reject, prior_sigma)
        self.schur = schur

    def _solve(self, H_, g, lam, n):
        N = H_.shape[0]
        if not self.schur:
            L = np.linalg.cholesky(H_ + lam * np.eye(N))
            return np.linalg.solve(L.T, np.linalg.solve(L, g))
        S = H_[:18, :18] + lam * np.eye(18)
        r = g[:18].copy()
        Ls, Ys, ygs = [], [], []
        for i in range(n):
            sl = slice(18 + 6 * i, 24 + 6 * i)
            Lc = np.linalg.cholesky(H_[sl, sl] + lam * np.eye(6))
            W = H_[sl, :18]
            Y = np.linalg.solve(Lc.T, np.linalg.solve(Lc, W))
            yg = np.linalg.solve(Lc.T, np.linalg.solve(Lc, g[sl]))
            S -= W.T @ Y
            r -= W.T @ yg
            Ls.append(Lc)
        Lx = np.linalg.cholesky(S)
        dx = np.linalg.solve(Lx.T, np.linalg.solve(Lx, r))
        out = [dx]
        for i in range(n):
            sl = slice(18 + 6 * i, 24 + 6 * i)
            rhs = g[sl] - H_[sl, :18] @ dx
            out.append(np.linalg.solve(Ls[i].T, np.linalg.solve(Ls[i], rhs)))
        return np.concatenate(out)

    # ---- problem evaluation ----
    def factors(self, pb, X1, X2, H, P1, P2):
        """yields (rows: whitened+reweighted r, {var: J}) per factor, in graph order"""
        out = []
        for X, Z, v in ((X1, pb.prior1, 0), (X2, pb.prior2, 1)):
            r = prior(X, Z) / self.sprior
            out.append(("prior", r, {v: np.eye(6) / self.sprior}))
        for i in range(len(P1)):
            for X, P, kp, vx, vp in ((X1, P1[i], pb.kp1[i], 0, 3 + 2 * i), (X2, P2[i], pb.kp2[i], 1, 4 + 2 * i)):
                r, Jx, Jp = project(X, P, pb.K, kp)
                r, Jx, Jp = r / self.sp, Jx / self.sp, Jp / self.sp
                w = np.sqrt(huber_w(np.linalg.norm(r), self.k))
                out.append(("proj", r * w, {vx: Jx * w, vp: Jp * w}, np.linalg.norm(r)))
            if pb.active[i]:
                r, J1, J2, J3 = ternary(P1[i], P2[i], H)
                r, J1, J2, J3 = r / self.sm, J1 / self.sm, J2 / self.sm, J3 / self.sm
                w = np.sqrt(huber_w(np.linalg.norm(r), self.k))
                out.append(("tern", r * w, {3 + 2 * i: J1 * w, 4 + 2 * i: J2 * w, 2: J3 * w}, np.linalg.norm(r)))
        return out

    def error(self, pb, X1, X2, H, P1, P2):
        e = 0.0
        for X, Z in ((X1, pb.prior1), (X2, pb.prior2)):
            r = prior(X, Z) / self.sprior
            e += 0.5 * (r @ r)
        for i in range(len(P1)):
            for X, P, kp in ((X1, P1[i], pb.kp1[i]), (X2, P2[i], pb.kp2[i])):
                r = project(X, P, pb.K, kp)[0] / self.sp
                e += huber_rho(np.linalg.norm(r), self.k)
            if pb.active[i]:
                r = ternary(P1[i], P2[i], H)[0] / self.sm
                e += huber_rho(np.linalg.norm(r), self.k)
        return e

    # ---- LM (GTSAM 4.2 LevenbergMarquardtOptimizer, oracle/oracle.c) ----
    def optimize(self, pb, max_iterations=100, lambda_initial=1e-5):
        n = len(pb.P1)
        dims = [6, 6, 6] + [3] * (2 * n)
        off = np.concatenate([[0], np.cumsum(dims)])
        N = off[-1]
        state = (pb.X1, pb.X2, pb.H, pb.P1.copy(), pb.P2.copy())
        err = self.error(pb, *state)
        err0 = err
        lam = lambda_initial
        it = inner = 0
        converged = False
        trace = []
        history = []  # (state, lambda) at the start of every outer iteration
        while True:
            history.append((state, lam))
            cur = err
            # iterate(): linearise once
            fs = self.factors(pb, *state)
            rows = sum(f[1].shape[0] for f in fs)
            A = np.zeros((rows, N))
            b = np.zeros(rows)
            r0 = 0
            for f in fs:
                m = f[1].shape[0]
                for v, J in f[2].items():
                    A[r0:r0 + m, off[v]:off[v] + dims[v]] = J
                b[r0:r0 + m] = -f[1]
                r0 += m
            H_ = A.T @ A
            g = A.T @ b
            oldLin = 0.5 * (b @ b)
            while True:
                step_ok = stop = False
                newErr = np.inf
                try:
                    delta = self._solve(H_, g, lam, n)
                    solved = True
                except np.linalg.LinAlgError:
                    solved = False
                if solved:
                    res = A @ delta - b
                    newLin = 0.5 * (res @ res)
                    linChange = oldLin - newLin
                    if linChange >= 0:
                        X1 = retract(state[0], delta[0:6])
                        X2 = retract(state[1], delta[6:12])
                        Hn = retract(state[2], delta[12:18])
                        d = delta[18:].reshape(n, 2, 3)
                        cand = (X1, X2, Hn, state[3] + d[:, 0], state[4] + d[:, 1])
                        newErr = self.error(pb, *cand)
                        costChange = err - newErr
                        if linChange > EPS * oldLin:
                            step_ok = costChange / linChange > 1e-3
                        if abs(costChange) < 1e-5 * err:
                            stop = True
                trace.append(dict(lam=lam, solved=solved, accepted=step_ok, new_error=newErr))
                if step_ok:
                    state, err = cand, newErr
                    lam /= 10.0
                    it += 1
                    inner += 1
                    break
                elif not stop:
                    lam *= 10.0
                    inner += 1
                    if lam >= 1e5:
                        break
                else:
                    break
            new = err
            converged = (new <= 0.0) or ((cur - new) / cur <= 1e-5) or (cur - new <= 1e-5)
            if not (it < max_iterations and not converged and np.isfinite(cur)):
                break
        history.append((state, lam))
        return dict(state=state, iterations=it, inner_iterations=inner, error_before=err0, error_after=err,
                    trace=trace, history=history)

    def outliers(self, pb, state):
        """determineFactorOutliers<LandmarkMotionTernaryFactor>: Gaussian error
        (robust model stripped) > 0.5 chi2(3, 0.99)"""
        thr = 0.5 * CHI2_3_099
        X1, X2, H, P1, P2 = state
        out = []
        for i in range(len(P1)):
            if not pb.active[i]:
                continue
            r = ternary(P1[i], P2[i], H)[0] / self.sm
            if 0.5 * (r @ r) > thr:
                out.append(i)
        return out

    def refine(self, pb):
        """MotionOnlyRefinementOptimizer::optimize (ProjectionError)."""
        res = self.optimize(pb)
        outl = self.outliers(pb, res["state"])
        res["status"] = OK
        res["outliers"] = []
        if outl and self.outlier_reject == 1:
            res["status"] = VALUES_KEY_EXISTS      # values.insert(motion key) throws
            res["outliers"] = list(outl)           # the detected ones, flagged
            return res
        if outl and self.outlier_reject == 2:
            rejected = set()
            for _ in range(4):
                for i in outl:
                    pb.active[i] = False
                    rejected.add(i)
                start = res["state"]
                pb.X1, pb.X2, pb.H = start[0], start[1], start[2]
                pb.P1, pb.P2 = start[3].copy(), start[4].copy()
                r2 = self.optimize(pb)
                res.update(state=r2["state"], error_after=r2["error_after"],
                           iterations=res["iterations"] + r2["iterations"],
                           inner_iterations=res["inner_iterations"] + r2["inner_iterations"])
                outl = self.outliers(pb, res["state"])
                if not outl:
                    break
            res["outliers"] = sorted(rejected)
        return res
