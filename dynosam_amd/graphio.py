"""The reference's dynosam graph-file format: reader and writer.

Mirrors NonlinearFactorGraphManager::writeDynosamGraphFile
(FactorGraphTools.cc:318-381) together with its serialisers:
  - factor lines: `TAG key... <measurement> <information, upper triangle>`
    (seralizeFactorToGraphFileFormat, FactorGraphTools.hpp:414-428;
    saveMatrixAsUpperTriangular, Numerical.hpp:276-294);
  - value lines: `TAG key <value>` (FactorGraphTools.hpp:431-438), written
    the first time a factor references the key.
Point3 values are `x y z`. Pose3 values are `x y z qx qy qz qw`
(toGraphFileFormat<Pose3>, FactorGraphTools.cc:262-267).

Reference tags: SE3_PRIOR_FACTOR, SE3_BETWEEN_FACTOR, SE3_MOTION_FACTOR
(LandmarkMotionTernaryFactor, measurement written as 0 0 0) and
POSE_TO_POINT_FACTOR; SE3_POSE_VALUE, SE3_MOTION_VALUE,
POINT3_STATIC_VALUE and POINT3_DYNAMIC_VALUE.

Extensions:
  - `HUBER <k>` at the end of a factor line. The reference writer casts
    every noise model to Gaussian, so it cannot write robust factors
    (FactorGraphTools.cc:275-277,305-307);
  - LANDMARK_MOTION_POSE_FACTOR (4 keys, `0 0 0`, 3x3 information) and
    LANDMARK_POSE_SMOOTHING_FACTOR (3 keys, no measurement, 6x6
    information) for the LLWorld formulation, plus SE3_OBJECT_POSE_VALUE.
Only diagonal information matrices are accepted. The device ABI takes
per-row sigmas, as the reference's Isotropic/Diagonal models do.

The writer uses round-trip precision (repr). The reference streams with
the default 6 significant digits, and the reader accepts both.
"""
import numpy as np

from . import _abi
from .graph import NonlinearFactorGraph, Values

# factor tag -> (factor type, n keys, measurement kind, information dim)
_FACTOR_TAGS = {
    "SE3_PRIOR_FACTOR": ("prior", 1, "pose", 6),
    "SE3_BETWEEN_FACTOR": ("between", 2, "pose", 6),
    "SE3_MOTION_FACTOR": ("landmark_motion_ternary", 3, "zero3", 3),
    "POSE_TO_POINT_FACTOR": ("pose_to_point", 2, "point", 3),
    "LANDMARK_MOTION_POSE_FACTOR": ("landmark_motion_pose", 4, "zero3", 3),
    "LANDMARK_POSE_SMOOTHING_FACTOR": ("landmark_pose_smoothing", 3, "none", 6),
}
_TYPE_TAG = {v[0]: k for k, v in _FACTOR_TAGS.items()}
# key character -> value tag (DynoChrExtractor cases, FactorGraphTools.cc:352-367)
_VALUE_TAGS = {
    "X": ("SE3_POSE_VALUE", _abi.POSE3),
    "H": ("SE3_MOTION_VALUE", _abi.POSE3),
    "l": ("POINT3_STATIC_VALUE", _abi.POINT3),
    "m": ("POINT3_DYNAMIC_VALUE", _abi.POINT3),
    "L": ("SE3_OBJECT_POSE_VALUE", _abi.POSE3),
}
_VALUE_KIND = {tag: kind for tag, kind in _VALUE_TAGS.values()}


class GraphFileError(ValueError):
    pass


def quat_to_rot(qx, qy, qz, qw):
    """Unit quaternion -> rotation matrix (gtsam::Rot3::Quaternion)."""
    n = np.sqrt(qx * qx + qy * qy + qz * qz + qw * qw)
    x, y, z, w = qx / n, qy / n, qz / n, qw / n
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
        [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
        [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)],
    ])


def rot_to_quat(R):
    """Rotation matrix -> (qx, qy, qz, qw) with qw >= 0 (Eigen's branch order)."""
    R = np.asarray(R, dtype=np.float64).reshape(3, 3)
    tr = R[0, 0] + R[1, 1] + R[2, 2]
    if tr > 0:
        s = np.sqrt(tr + 1.0) * 2
        q = [(R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s, 0.25 * s]
    elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        s = np.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
        q = [0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s, (R[2, 1] - R[1, 2]) / s]
    elif R[1, 1] > R[2, 2]:
        s = np.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
        q = [(R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s, (R[0, 2] - R[2, 0]) / s]
    else:
        s = np.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
        q = [(R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s, (R[1, 0] - R[0, 1]) / s]
    q = np.array(q)
    return q if q[3] >= 0 else -q


def _pose12(tokens):
    x, y, z, qx, qy, qz, qw = (float(t) for t in tokens)
    return np.concatenate([quat_to_rot(qx, qy, qz, qw).reshape(9), [x, y, z]])


def _pose_tokens(p12):
    p12 = np.asarray(p12, dtype=np.float64)
    q = rot_to_quat(p12[:9])
    return [repr(float(v)) for v in (p12[9], p12[10], p12[11], q[0], q[1], q[2], q[3])]


def _sigmas_from_info(tokens, dim, tag):
    vals = [float(t) for t in tokens]
    if len(vals) != dim * (dim + 1) // 2:
        raise GraphFileError(f"{tag}: expected {dim * (dim + 1) // 2} information entries, got {len(vals)}")
    info = np.zeros((dim, dim))
    k = 0
    for i in range(dim):
        for j in range(i, dim):
            info[i, j] = vals[k]
            k += 1
    off = info - np.diag(np.diag(info))
    if np.any(off != 0.0):
        raise GraphFileError(f"{tag}: only diagonal information matrices are supported")
    d = np.diag(info)
    if np.any(d <= 0.0):
        raise GraphFileError(f"{tag}: information must be positive")
    return 1.0 / np.sqrt(d)


def _info_tokens(sigmas, dim):
    s = np.broadcast_to(np.asarray(sigmas, dtype=np.float64), (dim,))
    out = []
    for i in range(dim):
        for j in range(i, dim):
            out.append(repr(float(1.0 / (s[i] * s[i]))) if i == j else "0")
    return out


def read(path_or_lines):
    """Parse a graph file -> (NonlinearFactorGraph, Values)."""
    lines = open(path_or_lines).read().splitlines() if isinstance(path_or_lines, str) else list(path_or_lines)
    graph = NonlinearFactorGraph()
    values = Values()
    seen = set()
    for ln, line in enumerate(lines, 1):
        tok = line.split()
        if not tok:
            continue
        tag = tok[0]
        if tag in _FACTOR_TAGS:
            ftype, nk, mkind, dim = _FACTOR_TAGS[tag]
            keys = [int(t) for t in tok[1:1 + nk]]
            rest = tok[1 + nk:]
            huber = 0.0
            if len(rest) >= 2 and rest[-2] == "HUBER":
                huber = float(rest[-1])
                rest = rest[:-2]
            nm = {"pose": 7, "point": 3, "zero3": 3, "none": 0}[mkind]
            meas = rest[:nm]
            sig = _sigmas_from_info(rest[nm:], dim, f"line {ln} {tag}")
            if ftype == "prior":
                graph.add_prior(keys[0], _pose12(meas), sig, huber)
            elif ftype == "between":
                graph.add_between(keys[0], keys[1], _pose12(meas), sig, huber)
            elif ftype == "pose_to_point":
                graph.add_pose_to_point(keys[0], keys[1], [float(t) for t in meas], sig, huber)
            elif ftype == "landmark_motion_ternary":
                graph.add_landmark_motion_ternary(keys[0], keys[1], keys[2], sig, huber)
            elif ftype == "landmark_motion_pose":
                graph.add_landmark_motion_pose(keys[0], keys[1], keys[2], keys[3], sig, huber)
            else:
                graph.add_landmark_pose_smoothing(keys[0], keys[1], keys[2], sig, huber)
        elif tag in _VALUE_KIND:
            key = int(tok[1])
            if key in seen:
                raise GraphFileError(f"line {ln}: value {key} written twice")
            seen.add(key)
            if _VALUE_KIND[tag] == _abi.POSE3:
                values.insert_pose(key, _pose12(tok[2:9]))
            else:
                values.insert_point(key, [float(t) for t in tok[2:5]])
        else:
            raise GraphFileError(f"line {ln}: unknown tag {tag!r}")
    return graph, values


def write(path, graph, values):
    """Write in the reference layout: each factor, then the values of the
    keys it introduces (first use). Factors are written grouped by type,
    in the order they were added within each type."""
    index = {int(k): i for i, k in enumerate(values.keys)}
    off = values._offsets()
    seen = set()
    out = []
    for ftype, (keys, meas, sig, hub) in graph.arrays().items():
        tag = _TYPE_TAG[ftype]
        _, nk, mkind, dim = _FACTOR_TAGS[tag]
        for f in range(keys.shape[0]):
            tok = [tag] + [str(int(k)) for k in keys[f]]
            if mkind == "pose":
                tok += _pose_tokens(meas[f])
            elif mkind == "point":
                tok += [repr(float(v)) for v in meas[f]]
            elif mkind == "zero3":
                tok += ["0", "0", "0"]
            tok += _info_tokens(sig[f], dim)
            if hub[f] > 0.0:
                tok += ["HUBER", repr(float(hub[f]))]
            out.append(" ".join(tok))
            for k in keys[f]:
                k = int(k)
                if k in seen:
                    continue
                seen.add(k)
                if k not in index:
                    raise GraphFileError(f"factor {tag} references key {k} with no value")
                i = index[k]
                chr_ = chr(k >> 56)
                if chr_ not in _VALUE_TAGS:
                    raise GraphFileError(f"key {k}: not a dynosam key (chr {chr_!r})")
                vtag, kind = _VALUE_TAGS[chr_]
                data = values.data[off[i]:off[i + 1]]
                vt = _pose_tokens(data) if kind == _abi.POSE3 else [repr(float(v)) for v in data]
                out.append(" ".join([vtag, str(k)] + vt))
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")
