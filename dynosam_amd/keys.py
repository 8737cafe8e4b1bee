"""dynosam key helpers (BackendDefinitions.hpp:57-88, BackendDefinitions.cc:35-61,
DynamicPointSymbol.cc:31-57), bound to the bit-exact C implementations in
libdynohip.so (host-only functions: no device needed)."""
import ctypes as C

from . import _native


def _lib():
    return _native.load("libdynohip.so")


def camera_pose_key(frame):
    """CameraPoseSymbol(k) = Symbol('X', k)."""
    return int(_lib().dynohip_camera_pose_key(int(frame)))


def static_landmark_key(tracklet):
    """StaticLandmarkSymbol(i) = Symbol('l', i)."""
    return int(_lib().dynohip_static_landmark_key(int(tracklet)))


def dynamic_landmark_key(frame, tracklet):
    """DynamicLandmarkSymbol(k, i) = Symbol('m', Cantor(i, k)); tracklet -1 is rejected."""
    k = C.c_uint64()
    if _lib().dynohip_dynamic_landmark_key(int(frame), int(tracklet), C.byref(k)) != 0:
        raise ValueError(f"invalid tracklet id {tracklet}")
    return int(k.value)


def object_motion_key(label, frame):
    """ObjectMotionSymbol(j, k) = LabeledSymbol('H', '0' + j, k)."""
    return int(_lib().dynohip_object_motion_key(int(label), int(frame)))


def object_pose_key(label, frame):
    """ObjectPoseSymbol(j, k) = LabeledSymbol('L', '0' + j, k)."""
    return int(_lib().dynohip_object_pose_key(int(label), int(frame)))
