"""LevenbergMarquardtOptimizer over the dynohip C-ABI (HIP on MI355X).

Python mirror of the reference call sites
    gtsam::LevenbergMarquardtOptimizer problem(graph, theta, opt_params);
    gtsam::Values optimised = problem.optimize();
    problem.iterations(); problem.getInnerIterations();
(RGBDBackendModule.cc:207-231, :364-383). The work runs in libdynohip.so;
there is no CPU fallback: a missing library or device raises.
"""
import ctypes as C

import numpy as np

from . import _abi, _native
from .graph import Values


class DynohipError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"dynohip error {code}: {msg}")
        self.code = code


def _check(lib, h, rc):
    if rc != 0:
        msg = lib.dynohip_last_error(h).decode() if h else ""
        raise DynohipError(rc, msg)


class Solver:
    """One dynohip_solver handle bound to a HIP device."""

    def __init__(self, device=0):
        self.lib = _native.load("libdynohip.so")
        self.h = C.c_void_p()
        rc = self.lib.dynohip_create(int(device), C.byref(self.h))
        if rc != 0:
            raise DynohipError(rc, "dynohip_create failed (no HIP device?)")
        self._graph = None
        self._values = None

    def close(self):
        if getattr(self, "h", None):
            self.lib.dynohip_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def set_graph(self, graph):
        self._graph = graph
        gv = graph.view()
        _check(self.lib, self.h, self.lib.dynohip_set_graph(self.h, C.byref(gv)))

    def set_values(self, values):
        self._values = values
        keys = np.ascontiguousarray(values.keys, dtype=np.uint64)
        kinds = np.ascontiguousarray(values.kinds, dtype=np.uint8)
        data = np.ascontiguousarray(values.data, dtype=np.float64)
        _check(self.lib, self.h, self.lib.dynohip_set_values(
            self.h, keys.ctypes.data_as(C.POINTER(C.c_uint64)), kinds.ctypes.data_as(C.POINTER(C.c_uint8)),
            data.ctypes.data_as(C.POINTER(C.c_double)), keys.shape[0]))

    def set_exec_options(self, wide_updates=256, level_backward=False, level_factor=False):
        """Execution paths (dynohip_set_exec_options): level-launched
        factorisation instead of the one-launch dataflow, and on that path a
        concurrent update kernel for levels with more than `wide_updates`
        update tasks; level-launched backward substitution."""
        _check(self.lib, self.h, self.lib.dynohip_set_exec_options(
            self.h, int(wide_updates), int(bool(level_backward)), int(bool(level_factor))))

    def values_data(self):
        n = self._values.data.shape[0]
        out = np.zeros(n)
        _check(self.lib, self.h, self.lib.dynohip_get_values(self.h, out.ctypes.data_as(C.POINTER(C.c_double)), n))
        return out

    def values(self):
        return self._values.with_data(self.values_data())

    def error(self):
        e = C.c_double()
        _check(self.lib, self.h, self.lib.dynohip_graph_error(self.h, C.byref(e)))
        return e.value

    def reset(self, params=None):
        params = params or _abi.LMParams.gtsam_default()
        _check(self.lib, self.h, self.lib.dynohip_lm_reset(self.h, C.byref(params)))

    def iterate(self):
        s = _abi.LMSummary()
        _check(self.lib, self.h, self.lib.dynohip_iterate(self.h, C.byref(s)))
        return s

    def optimize(self, params=None):
        params = params or _abi.LMParams.gtsam_default()
        s = _abi.LMSummary()
        _check(self.lib, self.h, self.lib.dynohip_optimize(self.h, C.byref(params), C.byref(s)))
        return s

    def trace(self):
        n = C.c_size_t()
        self.lib.dynohip_get_trace(self.h, None, 0, C.byref(n))
        arr = (_abi.TraceEntry * max(1, n.value))()
        self.lib.dynohip_get_trace(self.h, arr, n.value, C.byref(n))
        return _abi.trace_to_dicts(arr[: n.value])

    def solve_delta(self, lam):
        """Test hook: one damped solve at the current values and lambda
        (one tryLambda's linear system); returns (solved, delta) with delta
        in value order, 6 per pose and 3 per point."""
        kinds = self._values.kinds
        n = int(np.where(kinds == _abi.POSE3, 6, 3).sum())
        out = np.zeros(n)
        ok = C.c_int()
        _check(self.lib, self.h, self.lib.dynohip_solve_delta(self.h, float(lam),
                                                              out.ctypes.data_as(C.POINTER(C.c_double)), n,
                                                              C.byref(ok)))
        return bool(ok.value), out

    def linearize(self):
        n = self.lib.dynohip_linearize_size(self.h)
        out = np.zeros(n)
        _check(self.lib, self.h, self.lib.dynohip_linearize(self.h, out.ctypes.data_as(C.POINTER(C.c_double)), n))
        return out

    def stats(self):
        st = _abi.Stats()
        _check(self.lib, self.h, self.lib.dynohip_get_stats(self.h, C.byref(st)))
        return st.as_dict()

    def set_timing(self, enabled=True):
        _check(self.lib, self.h, self.lib.dynohip_set_timing(self.h, 1 if enabled else 0))

    def snapshot(self):
        _check(self.lib, self.h, self.lib.dynohip_values_snapshot(self.h))

    def restore(self):
        _check(self.lib, self.h, self.lib.dynohip_values_restore(self.h))


class LevenbergMarquardtOptimizer:
    """gtsam::LevenbergMarquardtOptimizer(graph, values, params) on the GPU."""

    def __init__(self, graph, values, params=None, device=0, solver=None):
        self.params = params or _abi.LMParams.gtsam_default()
        self.solver = solver or Solver(device)
        self.solver.set_graph(graph)
        self.solver.set_values(values)
        self._summary = None

    def optimize(self):
        self._summary = self.solver.optimize(self.params)
        return self.solver.values()

    def iterate(self):
        self._summary = self.solver.iterate()
        return self._summary

    def iterations(self):
        return self._summary.iterations if self._summary else 0

    def getInnerIterations(self):  # noqa: N802 (reference API name)
        return self._summary.inner_iterations if self._summary else 0

    def error(self):
        return self.solver.error()

    def summary(self):
        return self._summary

    def trace(self):
        return self.solver.trace()


def set_tile_ordering(leaf):
    """Tile ordering for plans built afterwards (process-wide): -1 automatic,
    0 frame order (plain band), k > 0 nested dissection with k-tile leaves."""
    _native.load("libdynohip.so").dynohip_set_tile_ordering(int(leaf))


def plan_schedule(graph, values):
    """Host-only: the tile Cholesky schedule the solver would run for this
    graph and key set (dynohip_plan_schedule). Returns a dict of arrays."""
    lib = _native.load("libdynohip.so")
    gv = graph.view()
    keys = np.ascontiguousarray(values.keys, dtype=np.uint64)
    kinds = np.ascontiguousarray(values.kinds, dtype=np.uint8)
    kp = keys.ctypes.data_as(C.POINTER(C.c_uint64))
    kk = kinds.ctypes.data_as(C.POINTER(C.c_uint8))
    info = _abi.ScheduleInfo()
    null = [None] * 12
    rc = lib.dynohip_plan_schedule(C.byref(gv), kp, kk, keys.shape[0], C.byref(info), *null)
    _check(lib, None, rc)
    shapes = {
        "tile_pos": info.n_tiles, "ftask": (info.n_ftask, 10), "pairs": (info.n_pairs, 2),
        "flevel": info.n_flevel,
        "btask": (info.n_btask, 4), "blevel": info.n_blevel, "bent": (info.n_bent, 2),
        "row_start": info.n_tiles + 1, "row_col": info.n_slots, "row_slot": info.n_slots,
        "red_a": info.n_red_blocks, "red_b": info.n_red_blocks,
    }
    arrs = {k: np.zeros(v, dtype=np.int32) for k, v in shapes.items()}
    ptrs = [arrs[k].ctypes.data_as(C.POINTER(C.c_int32)) for k in shapes]
    rc = lib.dynohip_plan_schedule(C.byref(gv), kp, kk, keys.shape[0], C.byref(info), *ptrs)
    _check(lib, None, rc)
    out = {k: getattr(info, k) for k, _ in _abi.ScheduleInfo._fields_}
    out.update(arrs)
    return out


def plan_export(graph, values, name, nranks=1, rank=0):
    """Host-only: one named int32 array of the (partitioned) plan of `rank`
    (dynohip_plan_export). Structs come back flattened: ftask and the
    separator phases' "phase<p>_ftask" 10 ints per task, bpart 8 ints per
    part."""
    lib = _native.load("libdynohip.so")
    gv = graph.view()
    keys = np.ascontiguousarray(values.keys, dtype=np.uint64)
    kinds = np.ascontiguousarray(values.kinds, dtype=np.uint8)
    kp = keys.ctypes.data_as(C.POINTER(C.c_uint64))
    kk = kinds.ctypes.data_as(C.POINTER(C.c_uint8))
    n = C.c_size_t()
    rc = lib.dynohip_plan_export(C.byref(gv), kp, kk, keys.shape[0], int(nranks), int(rank), name.encode(), None, 0,
                                 C.byref(n))
    _check(lib, None, rc)
    out = np.zeros(n.value, dtype=np.int32)
    rc = lib.dynohip_plan_export(C.byref(gv), kp, kk, keys.shape[0], int(nranks), int(rank), name.encode(),
                                 out.ctypes.data_as(C.POINTER(C.c_int32)), n.value, C.byref(n))
    _check(lib, None, rc)
    if name == "ftask" or (name.startswith("phase") and name.endswith("_ftask")):
        return out.reshape(-1, 10)
    if name == "bpart":
        return out.reshape(-1, 8)
    if name == "pairs":
        return out.reshape(-1, 2)
    return out
