"""TEST INFRASTRUCTURE — writer of frontend-output replay files in the
reference's format, to produce inputs for dynosam_amd.replay (the reader
under test). Restates:
  * nlohmann::json::to_bson (v3.11): objects as BSON documents with keys in
    std::map (sorted) order; arrays as documents keyed "0", "1", ...; doubles
    0x01; integers 0x10 when they fit int32 else 0x12; unsigned above int64
    0x11; strings 0x02; null 0x0A; bool 0x08;
  * nlohmann's std::map<non-string key, V> -> [[key, value], ...];
  * the reference's to_json for the packet (JsonUtils.cc:64-75), Pose3
    (JsonUtils.hpp:181-193, quaternion via Eigen), Eigen vectors
    (JsonUtils.hpp:155-164), MeasurementWithCovariance (:291-297),
    TrackedValueStatus (:322-330), ReferenceFrameValue (:277-280), the enums
    (:51-60) and GroundTruthInputPacket / ObjectPoseGT
    (GroundTruthPacket.cc:306-347);
  * JsonConverter::WriteBson: {"data": value} (Logger.hpp:193-204).
No file produced by the reference itself exists in this container (the OMD
replay is an external download), so the reader is pinned
against this restatement only: "parity unpinned" against real files.
"""
import struct
import sys
import os

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
from formulation import eigen_quaternion  # noqa: E402


class U64(int):
    """a FrameId (size_t): serialised as number_unsigned"""


def _cstr(s):
    return s.encode() + b"\x00"


def _element(name, v):
    if v is None:
        return b"\x0a" + _cstr(name)
    if isinstance(v, bool):
        return b"\x08" + _cstr(name) + (b"\x01" if v else b"\x00")
    if isinstance(v, U64):
        if v <= 2**31 - 1:
            return b"\x10" + _cstr(name) + struct.pack("<i", v)
        if v <= 2**63 - 1:
            return b"\x12" + _cstr(name) + struct.pack("<q", v)
        return b"\x11" + _cstr(name) + struct.pack("<Q", v)
    if isinstance(v, (int, np.integer)):
        v = int(v)
        if -2**31 <= v <= 2**31 - 1:
            return b"\x10" + _cstr(name) + struct.pack("<i", v)
        return b"\x12" + _cstr(name) + struct.pack("<q", v)
    if isinstance(v, (float, np.floating)):
        return b"\x01" + _cstr(name) + struct.pack("<d", float(v))
    if isinstance(v, str):
        b = v.encode()
        return b"\x02" + _cstr(name) + struct.pack("<i", len(b) + 1) + b + b"\x00"
    if isinstance(v, dict):
        return b"\x03" + _cstr(name) + _document(v)
    if isinstance(v, (list, tuple)):
        return b"\x04" + _cstr(name) + _document({str(i): x for i, x in enumerate(v)}, sort=False)
    raise TypeError(type(v))


def _document(d, sort=True):
    keys = sorted(d) if sort else list(d)
    body = b"".join(_element(k, d[k]) for k in keys)
    return struct.pack("<i", len(body) + 5) + body + b"\x00"


def to_bson(obj):
    assert isinstance(obj, dict), "to serialize to BSON, top-level type must be object"
    return _document(obj)


def pose_json(p12):
    q = eigen_quaternion(np.asarray(p12[:9]))
    return {"tx": float(p12[9]), "ty": float(p12[10]), "tz": float(p12[11]),
            "qx": float(q[0]), "qy": float(q[1]), "qz": float(q[2]), "qw": float(q[3])}


def eigen_json(v):
    return [[float(x)] for x in v]


def status_json(value, frame, tracklet, obj, rf="local"):
    return {"value": value, "frame_id": U64(frame), "tracklet_id": int(tracklet), "object_id": int(obj),
            "reference_frame": rf}


def packet_json(pk, keypoints=None, ground_truth=None):
    """RGBDInstanceOutputPacket -> json (JsonUtils.cc:64-75). keypoints: per
    measurement 2-D pixel (synthetic) or None for a projection."""
    def lists(meas):
        lm, kp = [], []
        for r in meas:
            z = np.asarray(r["landmark"], float)
            uv = [z[0] / z[2] * 500 + 320, z[1] / z[2] * 500 + 240] if z[2] != 0 else [0.0, 0.0]
            lm.append(status_json({"measurement": eigen_json(z)}, r["frame_id"], r["tracklet_id"], r["object_id"]))
            kp.append(status_json({"measurement": eigen_json(uv)}, r["frame_id"], r["tracklet_id"], r["object_id"]))
        return lm, kp

    st_l, st_k = lists(pk.static_measurements)
    dy_l, dy_k = lists(pk.dynamic_measurements)
    return {
        "frontend_type": "RGB",
        "static_keypoints": st_k,
        "dynamic_keypoints": dy_k,
        "T_world_camera": pose_json(pk.T_world_camera),
        "timestamp": float(pk.timestamp),
        "frame_id": U64(pk.frame_id),
        "ground_truth": ground_truth,
        "static_landmarks": st_l,
        "dynamic_landmarks": dy_l,
        "estimated_motions": [[int(o), {"estimate": pose_json(m), "reference_frame": "global"}]
                              for o, m in sorted(pk.estimated_motions.items())],
        "propogated_object_poses": [],
        "camera_poses": [pose_json(pk.T_world_camera)],
    }


def gt_json(frame, X12, objects, timestamp=0.0):
    """GroundTruthInputPacket (GroundTruthPacket.cc:306-347); objects:
    {object: (L_world12, prev_H_current_world12 or None)}"""
    objs = []
    for o, (L, H) in sorted(objects.items()):
        objs.append({"frame_id": U64(frame), "object_id": int(o), "L_camera": pose_json(L), "L_world": pose_json(L),
                     "bounding_box": {"x": 0, "y": 0, "width": 10, "height": 10}, "object_dimensions": None,
                     "prev_H_current_world": None if H is None else pose_json(H), "prev_H_current_L": None,
                     "prev_H_current_X": None, "motion_info": None})
    return {"timestamp": float(timestamp), "frame_id": U64(frame), "X_world": pose_json(X12), "objects": objs}


def write_frontend_output(path, packets, ground_truths=None):
    """JsonConverter::WriteOutJson(std::map<FrameId, RGBDInstanceOutputPacket>)"""
    data = [[U64(pk.frame_id), packet_json(pk, ground_truth=(ground_truths or {}).get(pk.frame_id))]
            for pk in sorted(packets, key=lambda p: p.frame_id)]
    blob = to_bson({"data": data})
    with open(path, "wb") as f:
        f.write(blob)
    return blob
