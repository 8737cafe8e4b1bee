"""Frontend-output replay: reads the BSON file the
reference frontend writes (std::map<FrameId, RGBDInstanceOutputPacket> through
JsonConverter::WriteOutJson, Logger.hpp:170-230) with the native reader in
libdynohip.so (dynosam_amd/csrc/replay.cpp), and yields the packets the
backend module consumes — the reference's offline path
(backend_experiments_node / FrontendPipeline replaying
rgbd_frontend_output.bson into RGBDBackendModule)."""
import ctypes as C

import numpy as np

from . import _abi, _native
from .backend import MEASUREMENT_DTYPE, BackendError, RGBDInstanceOutputPacket


def _lib():
    return _native.load("libdynohip.so")


class FrontendReplay:
    """Parsed replay file; packets in ascending frame order."""

    def __init__(self, path=None, data=None):
        self._lib = _lib()
        h = C.c_void_p()
        if data is not None:
            buf = np.frombuffer(bytes(data), dtype=np.uint8)
            rc = self._lib.dynob_replay_parse(buf.ctypes.data_as(C.POINTER(C.c_uint8)), buf.shape[0], C.byref(h))
        else:
            rc = self._lib.dynob_replay_open(str(path).encode(), C.byref(h))
        self._h = h
        if rc < 0:
            msg = self._lib.dynob_replay_last_error(h).decode() if h else ""
            raise BackendError(rc, msg)

    def __del__(self):
        if getattr(self, "_h", None):
            self._lib.dynob_replay_destroy(self._h)
            self._h = None

    def __len__(self):
        return int(self._lib.dynob_replay_num_packets(self._h))

    def packet(self, i):
        ip = _abi.InputPacket()
        rc = self._lib.dynob_replay_packet(self._h, i, C.byref(ip))
        if rc < 0:
            raise IndexError(i)

        def meas(ptr, n):
            if n == 0:
                return np.zeros(0, dtype=MEASUREMENT_DTYPE)
            raw = (C.c_uint8 * (n * MEASUREMENT_DTYPE.itemsize)).from_address(ptr)
            return np.frombuffer(raw, dtype=MEASUREMENT_DTYPE).copy()

        motions = {}
        for k in range(ip.n_motions):
            motions[int(ip.motion_object_ids[k])] = np.array(ip.motions12[12 * k:12 * k + 12])
        return RGBDInstanceOutputPacket(frame_id=int(ip.frame_id), T_world_camera=np.array(ip.T_world_camera[:]),
                                        static_measurements=meas(ip.static_measurements, ip.n_static),
                                        dynamic_measurements=meas(ip.dynamic_measurements, ip.n_dynamic),
                                        estimated_motions=motions, timestamp=float(ip.timestamp))

    def packets(self):
        return [self.packet(i) for i in range(len(self))]

    def ground_truth(self, i):
        """(X_world12, {object: (L_world12, prev_H_current_world12 or None)}) or None."""
        n = C.c_size_t()
        rc = self._lib.dynob_replay_ground_truth(self._h, i, None, None, None, None, 0, C.byref(n))
        if rc == 0:
            return None
        X = np.zeros(12)
        ids = np.zeros(n.value, dtype=np.int32)
        L = np.zeros((n.value, 12))
        H = np.zeros((n.value, 12))
        D = C.POINTER(C.c_double)
        self._lib.dynob_replay_ground_truth(self._h, i, X.ctypes.data_as(D), ids.ctypes.data_as(C.POINTER(C.c_int32)),
                                            L.ctypes.data_as(D), H.ctypes.data_as(D), n.value, C.byref(n))
        return X, {int(o): (L[k], None if np.isnan(H[k]).all() else H[k]) for k, o in enumerate(ids)}


def load_frontend_output(path):
    """Packets of a frontend-output replay file (e.g. rgbd_frontend_output.bson)."""
    return FrontendReplay(path).packets()
