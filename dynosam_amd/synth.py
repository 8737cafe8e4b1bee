"""Synthetic backend graphs via libdynosynth.so."""
import ctypes as C

import numpy as np

from . import _abi, _native
from .graph import NonlinearFactorGraph, Values

# SURVEY.md §8(d) / BASELINE.md configs (seed 42, backend.flags noise)
CONFIGS = {
    "C1": dict(frames=50, objects=1, static_landmarks=1460, dyn_slots=12),
    "C2": dict(frames=200, objects=3, static_landmarks=19200, dyn_slots=20),
    "NS": dict(frames=500, objects=5, static_landmarks=55000, dyn_slots=20),
    "C5": dict(frames=2000, objects=20, static_landmarks=320000, dyn_slots=10, object_visible_frames=1000),
    # small parity configs
    "T1": dict(frames=6, objects=1, static_landmarks=12, dyn_slots=2, dyn_track_len=4, static_track_len=3),
    "T2": dict(frames=20, objects=2, static_landmarks=120, dyn_slots=4),
}


def make_config(name=None, **overrides):
    lib = _native.load("libdynosynth.so")
    cfg = _abi.SynthConfig()
    lib.dynosynth_config_default(C.byref(cfg))
    params = dict(CONFIGS[name]) if name else {}
    params.update(overrides)
    for k, v in params.items():
        setattr(cfg, k, v)
    return cfg


def generate(name=None, **overrides):
    """Return (graph, values, ground_truth_data) for a named config."""
    lib = _native.load("libdynosynth.so")
    cfg = make_config(name, **overrides)
    h = C.c_void_p()
    rc = lib.dynosynth_generate(C.byref(cfg), C.byref(h))
    if rc != 0:
        raise ValueError(f"dynosynth_generate failed ({rc})")
    try:
        gv = _abi.GraphView()
        lib.dynosynth_graph(h, C.byref(gv))
        arrays = {}
        for i, t in enumerate(_abi.FACTOR_TYPES):
            blk = getattr(gv, t)
            n = blk.n
            nk, d, md = _abi.FACTOR_NKEYS[i], _abi.FACTOR_DIM[i], _abi.FACTOR_MEAS[i]
            if n == 0:
                arrays[t] = (np.zeros((0, nk), np.uint64), np.zeros((0, md), np.float64) if md else None,
                             np.zeros((0, d), np.float64), np.zeros(0, np.float64))
                continue
            keys = np.ctypeslib.as_array(blk.keys, shape=(n * nk,)).reshape(n, nk).copy()
            meas = np.ctypeslib.as_array(blk.measured, shape=(n * md,)).reshape(n, md).copy() if md else None
            sig = np.ctypeslib.as_array(blk.sigmas, shape=(n * d,)).reshape(n, d).copy()
            hub = np.ctypeslib.as_array(blk.huber_k, shape=(n,)).copy()
            arrays[t] = (keys, meas, sig, hub)
        nv = lib.dynosynth_num_values(h)
        nd = lib.dynosynth_values_len(h)
        keys = np.ctypeslib.as_array(lib.dynosynth_value_keys(h), shape=(nv,)).copy()
        kinds = np.ctypeslib.as_array(lib.dynosynth_value_kinds(h), shape=(nv,)).copy()
        data = np.ctypeslib.as_array(lib.dynosynth_value_data(h), shape=(nd,)).copy()
        gt = np.ctypeslib.as_array(lib.dynosynth_ground_truth(h), shape=(nd,)).copy()
    finally:
        lib.dynosynth_destroy(h)
    return NonlinearFactorGraph.from_arrays(arrays), Values(keys, kinds, data), gt
