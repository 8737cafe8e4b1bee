"""Sliding-window / full-batch drivers and window sharding across GPUs.

Reference behaviour (RGBDBackendModule.cc:235-245, 280-388;
RGBDBackendModule.hpp:87-145): windows are triggered by
SlidingWindow::check, every window is built with a *fresh* formulation
(initial theta deliberately unused, RGBDBackendModule.cc:288-300), solved
by an independent LM, and merged into the global theta with
Values::insert_or_assign in window order -- the last window wins
(Formulation-impl.hpp:53-60). Windows are therefore independent problems:
sharding them across ranks (one process per GPU) needs no data-path
collective, and merging the per-window results in window order reproduces
the serial result exactly.
"""
import ctypes as C

import numpy as np

from . import _abi, _native


class SlidingWindow:
    """RGBDBackendModule::SlidingWindow (C++ in libdynohip.so, bit-exact)."""

    def __init__(self, window=10, overlap=4):
        self._lib = _native.load("libdynohip.so")
        self._st = _abi.SlidingWindowState()
        self._lib.dynohip_sliding_window_init(C.byref(self._st), int(window), int(overlap))

    def check(self, frame_k):
        s, e = C.c_uint64(), C.c_uint64()
        cond = self._lib.dynohip_sliding_window_check(C.byref(self._st), int(frame_k), C.byref(s), C.byref(e))
        if cond < 0:
            # the reference's CHECK_GE (RGBDBackendModule.hpp:121-124, 139-141)
            raise ValueError(f"SlidingWindow::check({frame_k}): window start {ctypes_int(s.value)} before the "
                             f"first frame {self._st.first_frame}")
        return bool(cond), int(s.value), int(e.value)


def ctypes_int(u):
    """uint64 -> the int it was cast from."""
    return u - (1 << 64) if u >= (1 << 63) else u


def full_batch_trigger(full_batch_frame, frame_k):
    return bool(_native.load("libdynohip.so").dynohip_full_batch_trigger(int(full_batch_frame), int(frame_k)))


def window_schedule(first_frame, last_frame, window=10, overlap=4):
    """Windows [start, end] the reference backend optimises while spinning
    frames first_frame..last_frame. The bootstrap spin (the first frame)
    also calls check() (RGBDBackendModule.cc:148-149)."""
    sw = SlidingWindow(window, overlap)
    out = []
    for f in range(first_frame, last_frame + 1):
        cond, s, e = sw.check(f)
        if cond and f != first_frame:
            out.append((s, e))
    return out


def shard(n_windows, rank, world):
    """Contiguous block of window indices owned by `rank`."""
    base, rem = divmod(n_windows, world)
    start = rank * base + min(rank, rem)
    return list(range(start, start + base + (1 if rank < rem else 0)))


def merge_last_writer_wins(results):
    """Values::insert_or_assign in window order. `results` is an ordered
    list of (keys[uint64], kinds[uint8], data[float64]) per window."""
    theta = {}
    for keys, kinds, data in results:
        off = 0
        for k, kind in zip(keys, kinds):
            n = 12 if kind == _abi.POSE3 else 3
            theta[int(k)] = (int(kind), np.asarray(data[off:off + n], dtype=np.float64))
            off += n
    return theta
