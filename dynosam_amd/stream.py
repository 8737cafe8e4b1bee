"""Deterministic synthetic frontend output streams (RGBDInstanceOutputPacket
per frame) for the backend module.

The world follows SURVEY.md §8(d): a camera on a constant twist with a
random-walk frontend estimate, static landmarks tracked over consecutive
frames, and rigid objects on constant body twists carrying tracklets of
points. Per frame the packet holds the frontend camera pose, the static and
dynamic landmark measurements in the camera frame (z = X_k^-1 p + noise, the
3-D landmark of a LandmarkKeypoint) and noisy frontend object motions
(_{k-1}^wH_k). Tracklet ids: static 0..S-1, dynamic from S on; object labels
1..O (0 is the background label).

Feeding these packets through :class:`dynosam_amd.backend.RGBDBackendModule`
builds the reference graph for the stream (which factors, which first
observation is dropped, the min-observation and kMinNumberPoints gating).
"""
from dataclasses import dataclass

import numpy as np

from .backend import MEASUREMENT_DTYPE, RGBDInstanceOutputPacket


def _skew(w):
    return np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])


def expmap(xi):
    """Pose3::Expmap, tangent [w; v] -> 4x4."""
    w, v = np.asarray(xi[:3], float), np.asarray(xi[3:], float)
    th2 = w @ w
    T = np.eye(4)
    W = _skew(w)
    if th2 <= np.finfo(float).eps:
        T[:3, :3] = np.eye(3) + W
        T[:3, 3] = v
        return T
    th = np.sqrt(th2)
    K = W / th
    R = np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K
    T[:3, :3] = R
    wxv = np.cross(w, v)
    T[:3, 3] = (wxv - R @ wxv + w * (w @ v)) / th2
    return T


def inv(T):
    out = np.eye(4)
    out[:3, :3] = T[:3, :3].T
    out[:3, 3] = -T[:3, :3].T @ T[:3, 3]
    return out


def pose12(T):
    return np.concatenate([T[:3, :3].reshape(9), T[:3, 3]])


@dataclass
class StreamConfig:
    frames: int = 50
    objects: int = 1
    static_landmarks: int = 300
    static_track_len: int = 8
    dyn_slots: int = 12            # concurrent tracklets per object
    dyn_track_len: int = 10
    object_visible_frames: int = 0  # 0: visible throughout
    meas_noise: float = 0.01
    motion_noise: float = 0.01      # frontend motion estimate noise (rad / m)
    seed: int = 42
    # edge cases
    sparse_object_points: int = 0   # extra object with this many points per frame (< 3: never optimised)
    short_tracklets: int = 0        # dynamic tracklets of length 2 per object (< min_dynamic_obs)
    single_obs_static: int = 0      # static landmarks seen once (< min_static_obs)


def generate(cfg=StreamConfig()):
    """Returns (packets, ground_truth) with ground_truth = dict(X=[4x4],
    L={object: [4x4 per frame]}, static=xyz array)."""
    rng = np.random.default_rng(cfg.seed)
    F = cfg.frames
    step_c = expmap([0.01, 0.02, 0.005, 0.5, 0.0, 0.05])
    X = [np.eye(4)]
    Xfe = [np.eye(4)]
    for k in range(1, F):
        X.append(X[-1] @ step_c)
        n = np.concatenate([rng.normal(0, 0.005, 3), rng.normal(0, 0.02, 3)])
        Xfe.append(Xfe[-1] @ step_c @ expmap(n))
    meas = {k: {"static": [], "dynamic": []} for k in range(F)}

    # static landmarks: a track of consecutive frames around a world point
    S = cfg.static_landmarks
    Ls = min(cfg.static_track_len, F)
    starts = rng.integers(0, F - Ls + 1, size=S)
    local = np.stack([rng.normal(0, 6.0, S), rng.normal(0, 3.0, S), 12.0 + rng.normal(0, 4.0, S)], axis=1)
    static_world = np.zeros((S, 3))
    Xs = np.stack(X)                                        # F x 4 x 4
    mid = Xs[starts + Ls // 2]
    static_world = np.einsum("nij,nj->ni", mid[:, :3, :3], local) + mid[:, :3, 3]
    noise = rng.normal(0, cfg.meas_noise, (S, Ls, 3))
    for off in range(Ls):
        ks = starts + off
        Xk = Xs[ks]
        z = np.einsum("nji,nj->ni", Xk[:, :3, :3], static_world - Xk[:, :3, 3]) + noise[:, off]
        for i in range(S):
            meas[int(ks[i])]["static"].append((i, 0, z[i]))
    next_trk = S
    for j in range(cfg.single_obs_static):
        k = int(rng.integers(0, F))
        meas[k]["static"].append((next_trk, 0, rng.normal(0, 5.0, 3) + [0, 0, 10]))
        next_trk += 1

    # objects
    L = {}
    motions = {k: {} for k in range(F)}
    n_obj = cfg.objects + (1 if cfg.sparse_object_points else 0)
    for j in range(n_obj):
        label = j + 1
        v0, v1 = 0, F - 1
        if cfg.object_visible_frames and cfg.object_visible_frames < F:
            v0 = int(rng.integers(0, F - cfg.object_visible_frames + 1))
            v1 = v0 + cfg.object_visible_frames - 1
        xi = np.concatenate([rng.normal(0, 0.02, 3), [0.5 + rng.normal(0, 0.3)], rng.normal(0, 0.3, 2)])
        step_o = expmap(xi)
        L0 = np.eye(4)
        L0[:3, 3] = [rng.normal(0, 3.0), rng.normal(0, 1.0), 8.0 + rng.normal(0, 2.0)]
        Lj = [X[0] @ L0]
        for k in range(1, F):
            Lj.append(Lj[-1] @ step_o)
        L[label] = Lj
        for k in range(max(v0, 1), v1 + 1):
            H = Lj[k] @ inv(Lj[k - 1])
            noise = np.concatenate([rng.normal(0, cfg.motion_noise, 3), rng.normal(0, cfg.motion_noise, 3)])
            motions[k][label] = pose12(H @ expmap(noise))

        def add_tracklet(a, length):
            nonlocal next_trk
            trk = next_trk
            next_trk += 1
            body = rng.normal(0, 1.0, 3)
            for k in range(a, a + length):
                pw = Lj[k][:3, :3] @ body + Lj[k][:3, 3]
                z = X[k][:3, :3].T @ (pw - X[k][:3, 3]) + rng.normal(0, cfg.meas_noise, 3)
                meas[k]["dynamic"].append((trk, label, z))

        if j < cfg.objects:
            Ld = cfg.dyn_track_len
            slots = max(1, cfg.dyn_slots)
            for q in range(cfg.dyn_slots):
                a = v0 + (q * Ld) // slots
                while a + Ld - 1 <= v1:
                    add_tracklet(a, Ld)
                    a += Ld
            for _ in range(cfg.short_tracklets):
                add_tracklet(int(rng.integers(v0, max(v0 + 1, v1 - 1))), 2)
        else:  # the sparse object: a few points over its whole visibility
            for _ in range(cfg.sparse_object_points):
                add_tracklet(v0, v1 - v0 + 1)

    packets = []
    for k in range(F):
        st = meas[k]["static"]
        dy = meas[k]["dynamic"]

        def arr(items):
            a = np.zeros(len(items), dtype=MEASUREMENT_DTYPE)
            for i, (t, o, z) in enumerate(items):
                a[i]["tracklet_id"] = t
                a[i]["object_id"] = o
                a[i]["frame_id"] = k
                a[i]["landmark"] = z
            return a

        packets.append(RGBDInstanceOutputPacket(frame_id=k, T_world_camera=pose12(Xfe[k]), static_measurements=arr(st),
                                                dynamic_measurements=arr(dy), estimated_motions=dict(motions[k]),
                                                timestamp=0.05 * k))
    return packets, dict(X=X, L=L, static=static_world)
