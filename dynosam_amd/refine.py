"""Batched object-motion refinement on the GPU (include/dynorefine.h,
dynosam_amd/csrc/refine.hip) — MotionOnlyRefinementOptimizer::optimize
(ProjectionError) of dynosam/include/dynosam/frontend/vision/
MotionSolver-inl.hpp:277-470, for a whole batch of (object, frame pair)
problems in one kernel launch."""
import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _abi, _native
from .backend import BackendError

OK = 0
VALUES_KEY_EXISTS = 1


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


@dataclass
class RefineBatch:
    """Problems in CSR form over tracklets (host arrays)."""
    track_start: np.ndarray   # int32 (n + 1)
    X_k_1: np.ndarray         # (n, 12)
    X_k: np.ndarray           # (n, 12)
    H_init: np.ndarray        # (n, 12)
    calibration: np.ndarray   # (n, 5): fx, fy, s, u0, v0
    kp_k_1: np.ndarray        # (T, 2)
    kp_k: np.ndarray          # (T, 2)
    m_k_1: np.ndarray         # (T, 3)
    m_k: np.ndarray           # (T, 3)
    X_k_1_init: np.ndarray = None  # optional initial values (default: the priors)
    X_k_init: np.ndarray = None
    ternary_inactive: np.ndarray = None  # optional (T,) bool: ternaries out of the graph at the start

    @property
    def n(self):
        return int(self.track_start.shape[0] - 1)

    def problem(self, p):
        a, b = int(self.track_start[p]), int(self.track_start[p + 1])
        return dict(X_k_1=self.X_k_1[p], X_k=self.X_k[p], H=self.H_init[p], K=self.calibration[p],
                    kp_k_1=self.kp_k_1[a:b], kp_k=self.kp_k[a:b], m_k_1=self.m_k_1[a:b], m_k=self.m_k[a:b])


class MotionOnlyRefinementOptimizer:
    """MotionOnlyRefinementOptimizer with Params(landmark_motion_sigma 0.001,
    projection_sigma 2.0, k_huber 1e-4, outlier_reject true)."""

    def __init__(self, device=0, landmark_motion_sigma=0.001, projection_sigma=2.0, k_huber=0.0001,
                 outlier_reject=1, prior_sigma=1e-5):
        self._lib = _native.load("libdynohip.so")
        self.params = _abi.RefineParams(landmark_motion_sigma, projection_sigma, k_huber, prior_sigma,
                                        int(outlier_reject), 0)
        h = C.c_void_p()
        rc = self._lib.dynorefine_create(device, C.byref(h))
        if rc != 0:
            raise BackendError(rc, "dynorefine_create (no HIP device?)")
        self._h = h
        self._n = self._nt = 0

    def __del__(self):
        if getattr(self, "_h", None):
            self._lib.dynorefine_destroy(self._h)
            self._h = None

    def _check(self, rc):
        if rc != 0:
            raise BackendError(rc, self._lib.dynorefine_last_error(self._h).decode())

    def upload(self, batch):
        self._keep = [np.ascontiguousarray(a, dtype=np.float64) for a in
                      (batch.X_k_1, batch.X_k, batch.H_init, batch.calibration, batch.kp_k_1, batch.kp_k,
                       batch.m_k_1, batch.m_k)]
        ts = np.ascontiguousarray(batch.track_start, dtype=np.int32)
        self._keep.append(ts)
        inits = [None if a is None else np.ascontiguousarray(a, dtype=np.float64)
                 for a in (batch.X_k_1_init, batch.X_k_init)]
        self._keep += [a for a in inits if a is not None]
        inact = None
        if batch.ternary_inactive is not None:
            inact = np.ascontiguousarray(batch.ternary_inactive, dtype=np.uint8)
            assert inact.shape == (int(ts[-1]),)
            self._keep.append(inact)
        b = _abi.RefineBatch(batch.n, ts.ctypes.data_as(C.POINTER(C.c_int32)), *[_dp(a) for a in self._keep[:8]],
                             *[C.POINTER(C.c_double)() if a is None else _dp(a) for a in inits],
                             C.POINTER(C.c_uint8)() if inact is None else inact.ctypes.data_as(C.POINTER(C.c_uint8)))
        self._check(self._lib.dynorefine_upload(self._h, C.byref(b)))
        self._n, self._nt = batch.n, int(ts[-1])

    def solve(self, lm_params=None):
        lm = lm_params or _abi.LMParams.gtsam_default()
        self._check(self._lib.dynorefine_solve(self._h, C.byref(self.params), C.byref(lm)))
        return self._lib.dynorefine_last_solve_ms(self._h)

    def download(self):
        H = np.zeros((self._n, 12))
        out = np.zeros(max(self._nt, 1), dtype=np.uint8)
        res = (_abi.RefineResult * max(self._n, 1))()
        self._check(self._lib.dynorefine_download(self._h, _dp(H), out.ctypes.data_as(C.POINTER(C.c_uint8)), res))
        results = [{f: getattr(r, f) for f, _ in r._fields_} for r in res[:self._n]]
        return H, out[:self._nt].astype(bool), results

    def optimize_batch(self, batch, lm_params=None):
        """Returns (H (n x 12), outlier flags per tracklet, per-problem results)."""
        self.upload(batch)
        self.solve(lm_params)
        return self.download()


def _expmap(xi):
    w, v = np.asarray(xi[:3], float), np.asarray(xi[3:], float)
    th2 = w @ w
    W = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
    if th2 <= np.finfo(float).eps:
        return np.eye(3) + W, v.copy()
    th = np.sqrt(th2)
    K = W / th
    R = np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K
    wxv = np.cross(w, v)
    return R, (wxv - R @ wxv + w * (w @ v)) / th2


def synthetic_batch(n_problems=256, tracks=(20, 60), seed=0, outlier_frac=0.0, pixel_noise=0.5,
                    depth_noise=0.01, behind_camera=0):
    """Frontend-like problems: an object seen from X_{k-1} and X_k moving by
    H; keypoints are projections + noise, points are noisy back-projections
    (the frontend's backProjectToWorld), H_init is a perturbed motion.
    outlier_frac of the tracklets get a wrong point at k; `behind_camera`
    problems have one point behind the camera at k (CheiralityException)."""
    rng = np.random.default_rng(seed)
    counts = rng.integers(tracks[0], tracks[1] + 1, size=n_problems)
    ts = np.zeros(n_problems + 1, dtype=np.int32)
    ts[1:] = np.cumsum(counts)
    T = int(ts[-1])
    X1 = np.zeros((n_problems, 12))
    X2 = np.zeros((n_problems, 12))
    H0 = np.zeros((n_problems, 12))
    Kc = np.zeros((n_problems, 5))
    kp1 = np.zeros((T, 2))
    kp2 = np.zeros((T, 2))
    m1 = np.zeros((T, 3))
    m2 = np.zeros((T, 3))
    for p in range(n_problems):
        Ra, ta = _expmap(rng.normal(0, 0.2, 6))
        dR, dt = _expmap(np.concatenate([rng.normal(0, 0.02, 3), rng.normal(0, 0.1, 3)]))
        Rb, tb = Ra @ dR, Ra @ dt + ta
        HR, Ht = _expmap(np.concatenate([rng.normal(0, 0.05, 3), rng.normal(0, 0.3, 3)]))
        K = np.array([500.0 + rng.normal(0, 20), 500.0 + rng.normal(0, 20), 0.0, 320.0, 240.0])
        center = ta + Ra @ np.array([rng.normal(0, 1.0), rng.normal(0, 0.5), 8.0 + rng.normal(0, 2.0)])
        for i in range(ts[p], ts[p + 1]):
            pw1 = center + rng.normal(0, 1.0, 3)
            pw2 = HR @ pw1 + Ht
            if rng.random() < outlier_frac:
                pw2 = pw2 + rng.normal(0, 0.5, 3)
            for (R, t, pw, kp, m) in ((Ra, ta, pw1, kp1, m1), (Rb, tb, pw2, kp2, m2)):
                q = R.T @ (pw - t)
                u = K[0] * q[0] / q[2] + K[2] * q[1] / q[2] + K[3]
                v = K[1] * q[1] / q[2] + K[4]
                kp[i] = [u + rng.normal(0, pixel_noise), v + rng.normal(0, pixel_noise)]
                m[i] = pw + rng.normal(0, depth_noise, 3)
        if p < behind_camera and ts[p + 1] > ts[p]:
            m2[ts[p]] = tb - Rb @ np.array([0.0, 0.0, 2.0])  # 2 m behind the camera at k
        X1[p] = np.concatenate([Ra.reshape(9), ta])
        X2[p] = np.concatenate([Rb.reshape(9), tb])
        nR, nt = _expmap(np.concatenate([rng.normal(0, 0.01, 3), rng.normal(0, 0.05, 3)]))
        H0[p] = np.concatenate([(HR @ nR).reshape(9), HR @ nt + Ht])
        Kc[p] = K
    return RefineBatch(ts, X1, X2, H0, Kc, kp1, kp2, m1, m2)
