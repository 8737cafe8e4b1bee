"""ctypes binding of the CPU oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.
"""
import ctypes as C
import os

import numpy as np

from dynosam_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "build", "liboracle.so")
# the same restatement with glibc's sin / tan / acos (what GTSAM calls) in
# place of the shared trig.h: the independent check of trig.h's rounding
ORACLE_LIBM_SO = os.path.join(ROOT, "oracle", "build", "liboracle_libm.so")
_libs = {}


def lib(libm=False):
    if libm not in _libs:
        path = ORACLE_LIBM_SO if libm else ORACLE_SO
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C oracle`")
        L = C.CDLL(path)
        P = C.POINTER
        vp = C.c_void_p
        L.oracle_create.argtypes = [P(_abi.GraphView), P(C.c_uint64), P(C.c_uint8), P(C.c_double), C.c_size_t, P(vp)]
        L.oracle_create.restype = C.c_int
        L.oracle_destroy.argtypes = [vp]
        L.oracle_last_error.argtypes = [vp]
        L.oracle_last_error.restype = C.c_char_p
        L.oracle_set_dense.argtypes = [vp, C.c_int]
        L.oracle_set_reverse_sums.argtypes = [vp, C.c_int]
        L.oracle_set_reverse_sums.restype = None
        L.oracle_set_solve_ld.argtypes = [vp, C.c_int]
        L.oracle_set_solve_ld.restype = None
        L.oracle_set_threads.argtypes = [vp, C.c_int]
        L.oracle_set_threads.restype = C.c_int
        L.oracle_error.argtypes = [vp]
        L.oracle_error.restype = C.c_double
        L.oracle_lm_reset.argtypes = [vp, P(_abi.LMParams)]
        L.oracle_iterate.argtypes = [vp, P(_abi.LMSummary)]
        L.oracle_optimize.argtypes = [vp, P(_abi.LMParams), P(_abi.LMSummary)]
        L.oracle_get_values.argtypes = [vp, P(C.c_double), C.c_size_t]
        L.oracle_set_values_data.argtypes = [vp, P(C.c_double), C.c_size_t]
        L.oracle_get_trace.argtypes = [vp, P(_abi.TraceEntry), C.c_size_t, P(C.c_size_t)]
        L.oracle_linearize_size.argtypes = [vp]
        L.oracle_linearize_size.restype = C.c_size_t
        L.oracle_linearize.argtypes = [vp, P(C.c_double), C.c_size_t]
        L.oracle_solve_damped.argtypes = [vp, C.c_double, P(C.c_double), C.c_size_t]
        L.oracle_solve_damped_ld.argtypes = [vp, C.c_double, P(C.c_double), C.c_size_t]
        L.oracle_eval_factor.argtypes = [C.c_int, P(C.c_double), P(C.c_double), P(C.c_double), P(C.c_double)]
        for fn in ("oracle_factor_dim", "oracle_factor_cols", "oracle_factor_nkeys"):
            getattr(L, fn).argtypes = [C.c_int]
        for fn in ("oracle_pose_expmap", "oracle_pose_logmap", "oracle_rot_expmap", "oracle_rot_logmap", "oracle_pose_inverse"):
            getattr(L, fn).argtypes = [P(C.c_double), P(C.c_double)]
        L.oracle_pose_compose.argtypes = [P(C.c_double)] * 3
        L.oracle_cantor_pair.argtypes = [C.c_uint64, C.c_uint64]
        L.oracle_cantor_pair.restype = C.c_uint64
        L.oracle_cantor_depair.argtypes = [C.c_uint64, P(C.c_uint64), P(C.c_uint64)]
        L.oracle_symbol.argtypes = [C.c_ubyte, C.c_uint64]
        L.oracle_symbol.restype = C.c_uint64
        L.oracle_labeled_symbol.argtypes = [C.c_ubyte, C.c_ubyte, C.c_uint64]
        L.oracle_labeled_symbol.restype = C.c_uint64
        L.oracle_reconstruct_labeled.argtypes = [C.c_uint64, C.c_ubyte, P(C.c_int), P(C.c_uint64)]
        L.oracle_chr_extract.argtypes = [C.c_uint64]
        L.oracle_chr_extract.restype = C.c_ubyte
        _libs[libm] = L
    return _libs[libm]


def dptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class Oracle:
    """CPU restatement of LevenbergMarquardtOptimizer(graph, values).optimize()."""

    def __init__(self, graph, values, dense=False, threads=1, reverse_sums=False, libm=False, solve_ld=False):
        L = self.L = lib(libm)
        self.graph = graph
        self.values = values
        self._gv = graph.view()
        self.h = C.c_void_p()
        keys = np.ascontiguousarray(values.keys)
        kinds = np.ascontiguousarray(values.kinds)
        data = np.ascontiguousarray(values.data)
        rc = L.oracle_create(C.byref(self._gv), keys.ctypes.data_as(C.POINTER(C.c_uint64)),
                             kinds.ctypes.data_as(C.POINTER(C.c_uint8)), dptr(data), len(keys), C.byref(self.h))
        if rc != 0:
            msg = L.oracle_last_error(self.h).decode()
            L.oracle_destroy(self.h)
            self.h = None
            raise ValueError(f"oracle_create: {rc} {msg}")
        L.oracle_set_dense(self.h, 1 if dense else 0)
        if reverse_sums:
            L.oracle_set_reverse_sums(self.h, 1)
        if threads > 1:
            L.oracle_set_threads(self.h, int(threads))
        if solve_ld:   # every LM step solved in extended precision: the exact-step trajectory
            L.oracle_set_solve_ld(self.h, 1)
        self.ndata = data.shape[0]

    def __del__(self):
        if getattr(self, "h", None):
            self.L.oracle_destroy(self.h)
            self.h = None

    def error(self):
        return self.L.oracle_error(self.h)

    def optimize(self, params=None):
        params = params or _abi.LMParams.gtsam_default()
        s = _abi.LMSummary()
        self.L.oracle_optimize(self.h, C.byref(params), C.byref(s))
        return s

    def reset(self, params=None):
        params = params or _abi.LMParams.gtsam_default()
        self.L.oracle_lm_reset(self.h, C.byref(params))

    def iterate(self):
        s = _abi.LMSummary()
        self.L.oracle_iterate(self.h, C.byref(s))
        return s

    def values_data(self):
        out = np.zeros(self.ndata)
        self.L.oracle_get_values(self.h, dptr(out), self.ndata)
        return out

    def set_values_data(self, data):
        data = np.ascontiguousarray(data, dtype=np.float64)
        self.L.oracle_set_values_data(self.h, dptr(data), data.shape[0])

    def trace(self):
        n = C.c_size_t()
        self.L.oracle_get_trace(self.h, None, 0, C.byref(n))
        arr = (_abi.TraceEntry * max(1, n.value))()
        self.L.oracle_get_trace(self.h, arr, n.value, C.byref(n))
        return _abi.trace_to_dicts(arr[: n.value])

    def linearize(self):
        n = self.L.oracle_linearize_size(self.h)
        out = np.zeros(n)
        self.L.oracle_linearize(self.h, dptr(out), n)
        return out

    def solve_damped(self, lam):
        n = int((np.where(self.values.kinds == _abi.POSE3, 6, 3)).sum())
        out = np.zeros(n)
        ok = self.L.oracle_solve_damped(self.h, lam, dptr(out), n)
        return ok, out

    def solve_damped_ld(self, lam):
        """the same step with the Schur solve in extended precision (a
        reference for ill-conditioned systems)"""
        n = int((np.where(self.values.kinds == _abi.POSE3, 6, 3)).sum())
        out = np.zeros(n)
        ok = self.L.oracle_solve_damped_ld(self.h, lam, dptr(out), n)
        return ok, out


def eval_factor(ftype, vars_concat, meas=None):
    L = lib()
    d = L.oracle_factor_dim(ftype)
    cols = L.oracle_factor_cols(ftype)
    v = np.ascontiguousarray(vars_concat, dtype=np.float64)
    m = np.ascontiguousarray(meas, dtype=np.float64) if meas is not None else np.zeros(12)
    r = np.zeros(d)
    J = np.zeros(d * cols)
    L.oracle_eval_factor(ftype, dptr(v), dptr(m), dptr(r), dptr(J))
    return r, J.reshape(d, cols)


def pose_expmap(xi):
    out = np.zeros(12)
    lib().oracle_pose_expmap(dptr(np.ascontiguousarray(xi, dtype=np.float64)), dptr(out))
    return out


def pose_logmap(T):
    out = np.zeros(6)
    lib().oracle_pose_logmap(dptr(np.ascontiguousarray(T, dtype=np.float64)), dptr(out))
    return out


def pose_compose(A, B):
    out = np.zeros(12)
    lib().oracle_pose_compose(dptr(np.ascontiguousarray(A, dtype=np.float64)), dptr(np.ascontiguousarray(B, dtype=np.float64)), dptr(out))
    return out


def pose_inverse(A):
    out = np.zeros(12)
    lib().oracle_pose_inverse(dptr(np.ascontiguousarray(A, dtype=np.float64)), dptr(out))
    return out
