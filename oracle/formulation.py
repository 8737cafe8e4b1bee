"""TEST INFRASTRUCTURE — CPU restatement (pure Python) of the reference's
backend graph construction, the checker for dynosam_amd/csrc/backend.cpp.
Only tests/ may import it; the product never does.

Restates, line by line:
  Map::addOrUpdateMapStructures          Map.hpp:376-444
  FrameNode / LandmarkNode / ObjectNode   MapNodes-inl.hpp:37-262
  Formulation::setInitialPose / Prior     Formulation-impl.hpp:83-104
  Formulation::addOdometry                Formulation-impl.hpp:128-161
  Formulation::updateStaticObservations   Formulation-impl.hpp:203-305
  Formulation::updateDynamicObservations  Formulation-impl.hpp:307-584
  WorldMotionFormulation callbacks        WorldMotionEstimator.cc:155-316
  WorldPoseFormulation callbacks          WorldPoseEstimator.cc:84-286
  Accessor::computeObjectCentroid         Accessor-impl.hpp:290-318 (PCL
                                          CentroidPoint: float accumulation)
  RGBDBackendModule spin / constructGraph RGBDBackendModule.cc:129-296
  SlidingWindow::check                    RGBDBackendModule.hpp:115-144
Parity of this restatement against the reference itself is pinned by the
reference's Map tests (test_map.cc:43-392, restated in tests/test_backend.py);
the formulation's graph output has no reference fixture (the reference's
backend tests only write files), so beyond the Map pins it is "parity
unpinned" against the C++ reference and checked against this independent
restatement.
"""
import numpy as np

POSE_TO_POINT, TERNARY, BETWEEN, PRIOR, MOTION_POSE, POSE_SMOOTHING = range(6)


def symbol(c, j):
    return (ord(c) << 56) | (j & ((1 << 56) - 1))


def labeled(c, label, j):
    return (ord(c) << 56) | (label << 48) | (j & ((1 << 48) - 1))


def cantor(a, b):
    return (a + b) * (a + b + 1) // 2 + b


def X_key(f):
    return symbol("X", f)


def l_key(t):
    return symbol("l", t)


def m_key(f, t):
    return symbol("m", cantor(t, f))


def H_key(o, f):
    return labeled("H", ord("0") + o, f)


def L_key(o, f):
    return labeled("L", ord("0") + o, f)


def T_of(p12):
    T = np.eye(4)
    T[:3, :3] = np.asarray(p12[:9]).reshape(3, 3)
    T[:3, 3] = p12[9:12]
    return T


def p12_of(T):
    return np.concatenate([T[:3, :3].reshape(9), T[:3, 3]])


def inv(T):
    out = np.eye(4)
    out[:3, :3] = T[:3, :3].T
    out[:3, 3] = -T[:3, :3].T @ T[:3, 3]
    return out


def transform_from(T, p):
    return T[:3, :3] @ np.asarray(p) + T[:3, 3]


class Abort(RuntimeError):
    """A glog CHECK / LOG(FATAL) / thrown exception in the reference."""


class Map:
    def __init__(self):
        self.frames = {}      # frame -> dict(static=set, dynamic=set, objects=set, X=None, motions=None)
        self.landmarks = {}   # tracklet -> dict(object=int, meas={frame: xyz})
        self.objects = {}     # object -> set(tracklets)

    def add(self, trk, obj, frame, z):
        if trk not in self.landmarks:
            self.landmarks[trk] = dict(object=obj, meas={})
        fr = self.frames.setdefault(frame, dict(static=set(), dynamic=set(), objects=set(), X=None, motions=None))
        ln = self.landmarks[trk]
        if ln["object"] != obj:
            raise Abort("object label changed")
        if frame in ln["meas"]:
            raise Abort("duplicate measurement")
        ln["meas"][frame] = np.asarray(z, dtype=float)
        if obj == 0:
            fr["static"].add(trk)
        else:
            self.objects.setdefault(obj, set()).add(trk)
            fr["dynamic"].add(trk)
            fr["objects"].add(obj)

    def seen_frames(self, trk):
        return sorted(self.landmarks[trk]["meas"])

    def object_observed(self, f, o):
        return f in self.frames and o in self.frames[f]["objects"]

    def motion_expected(self, f, o):
        return self.object_observed(f, o) and self.object_observed(f - 1, o)

    def lmks_at(self, o, f):
        return sorted(t for t in self.objects.get(o, ()) if f in self.landmarks[t]["meas"])

    def object_seen_frames(self, o):
        s = set()
        for t in self.objects.get(o, ()):
            s |= set(self.landmarks[t]["meas"])
        return sorted(s)


class Formulation:
    def __init__(self, mp, formulation=0, min_static=2, min_dynamic=3, smoothing=True, init_H_identity=True,
                 noise=None):
        self.map = mp
        self.kind = formulation
        self.min_static, self.min_dynamic = min_static, min_dynamic
        self.smoothing, self.init_H_identity = smoothing, init_H_identity
        self.noise = noise
        self.theta = {}
        self.factors = []
        self.other_in_map = set()
        self.tracklet_in_map = set()

    def _factor(self, out, t, keys, meas, noise):
        out.append((t, tuple(keys), None if meas is None else np.asarray(meas, dtype=float), noise))

    def sensor_pose(self, f):
        return self.theta.get(X_key(f))

    def init_or_lin_pose(self, f):
        Xt = self.sensor_pose(f)
        if self.map.frames[f]["X"] is None:
            raise Abort("no initial sensor pose")
        return Xt if Xt is not None else self.map.frames[f]["X"]

    def set_initial_pose(self, f, T):
        self.theta[X_key(f)] = np.asarray(T, float)

    def set_initial_pose_prior(self, f, T):
        self._factor(self.factors, PRIOR, [X_key(f)], T, self.noise["prior"])

    def add_odometry(self, f, T):
        self.theta[X_key(f)] = np.asarray(T, float)
        Tk1 = self.map.frames[f - 1]["X"]
        odom = p12_of(inv(T_of(Tk1)) @ T_of(T))
        self._factor(self.factors, BETWEEN, [X_key(f - 1), X_key(f)], odom, self.noise["odometry"])

    def update_static(self, k, do_backtrack=False):
        Tfe = T_of(self.map.frames[k]["X"])
        for t in sorted(self.map.frames[k]["static"]):
            ln = self.map.landmarks[t]
            key = l_key(t)
            if key in self.other_in_map:
                self._factor(self.factors, POSE_TO_POINT, [X_key(k), key], ln["meas"][k], self.noise["static"])
                continue
            if len(ln["meas"]) < self.min_static:
                continue
            for s in self.map.seen_frames(t):
                if s > k:
                    break
                if not do_backtrack and s < k:
                    continue
                self._factor(self.factors, POSE_TO_POINT, [X_key(s), key], ln["meas"][s], self.noise["static"])
            v = self.theta.get(key)
            self.theta[key] = v if v is not None else transform_from(Tfe, ln["meas"][k])
            self.other_in_map.add(key)

    def _point_update(self, t, o, f1, f, Xk, Xk1, starting, affected, local):
        ln = self.map.landmarks[t]
        k1, kk = m_key(f1, t), m_key(f, t)
        if starting:
            if self.kind == 0 and k1 in self.theta:
                raise Abort("point at k-1 exists")
            self._factor(local["factors"], POSE_TO_POINT, [X_key(f1), k1], ln["meas"][f1], self.noise["dynamic"])
            affected.setdefault(o, set()).add(f1)
            v = self.theta.get(k1)
            local["values"][k1] = v if v is not None else transform_from(T_of(Xk1), ln["meas"][f1])
        if k1 not in local["values"] and k1 not in self.theta:
            raise Abort("previous point missing")
        self._factor(local["factors"], POSE_TO_POINT, [X_key(f), kk], ln["meas"][f], self.noise["dynamic"])
        affected.setdefault(o, set()).add(f)
        v = self.theta.get(kk)
        if kk in local["values"]:
            raise Abort("ValuesKeyAlreadyExists")
        local["values"][kk] = v if v is not None else transform_from(T_of(Xk), ln["meas"][f])
        if self.kind == 0:
            self._factor(local["factors"], TERNARY, [k1, kk, H_key(o, f)], None, self.noise["motion"])
        else:
            self._factor(local["factors"], MOTION_POSE, [k1, kk, L_key(o, f1), L_key(o, f)], None,
                         self.noise["motion"])
        affected[o] |= {f1, f}
        self.tracklet_in_map.add(t)

    def centroid(self, f, o):
        pts = []
        for t in sorted(self.map.frames[f]["dynamic"]):
            if self.map.landmarks[t]["object"] != o:
                continue
            v = self.theta.get(m_key(f, t))
            if v is not None:
                pts.append(v)
        if not pts:
            return None
        acc = np.zeros(3, dtype=np.float32)
        for p in pts:
            acc = (acc + np.asarray(p, dtype=np.float32)).astype(np.float32)
        return (acc / np.float32(len(pts))).astype(np.float64)

    def _object_update(self, f, o, has_pair, out_factors):
        if self.kind == 0:
            Hk = H_key(o, f)
            if not has_pair:
                return
            if Hk not in self.other_in_map:
                init = np.eye(4)
                if not self.init_H_identity:
                    mo = (self.map.frames[f]["motions"] or {}).get(o)
                    if mo is not None:
                        init[:3, 3] = np.asarray(mo)[9:12]
                self.theta[Hk] = p12_of(init)
                self.other_in_map.add(Hk)
            if f < 2 or (f - 1) not in self.map.frames:
                return
            if self.smoothing and self.map.object_observed(f - 1, o):
                Hk1 = H_key(o, f - 1)
                if Hk1 in self.other_in_map and Hk in self.other_in_map:
                    self._factor(out_factors, BETWEEN, [Hk1, Hk], p12_of(np.eye(4)), self.noise["smoothing"])
            return
        Lk = L_key(o, f)
        if Lk not in self.other_in_map:
            prev = self.theta.get(L_key(o, f - 1)) if (f - 1) in self.map.frames else None
            mo = (self.map.frames[f]["motions"] or {}).get(o)
            if mo is not None and prev is not None:
                pose = p12_of(T_of(mo) @ T_of(prev))
                if self.map.object_seen_frames(o)[0] == f:
                    raise Abort("motion at first seen frame")
            else:
                c = self.centroid(f, o)
                if c is None:
                    raise Abort("no centroid")
                init = np.eye(4)
                init[:3, 3] = c
                v = self.theta.get(Lk)
                pose = v if v is not None else p12_of(init)
            self.theta[Lk] = pose
            self.other_in_map.add(Lk)
        if self.smoothing:
            if f < 2 or (f - 2) not in self.map.frames or (f - 1) not in self.map.frames:
                return
            k2, k1 = L_key(o, f - 2), L_key(o, f - 1)
            if k1 in self.other_in_map and Lk in self.other_in_map and k2 in self.other_in_map:
                self._factor(out_factors, POSE_SMOOTHING, [k2, k1, Lk], None, self.noise["smoothing"])

    def update_dynamic(self, k, do_backtrack=False):
        out = []
        affected = {}
        for o in sorted(self.map.frames[k]["objects"]):
            if not self.map.motion_expected(k, o):
                continue
            seen_k = self.map.lmks_at(o, k)
            if len(seen_k) < 3 or len(self.map.lmks_at(o, k - 1)) < 3:
                continue
            for t in seen_k:
                if len(self.map.landmarks[t]["meas"]) < self.min_dynamic:
                    continue
                local = dict(values={}, factors=out)
                if t not in self.tracklet_in_map:
                    seen = self.map.seen_frames(t)
                    start = seen[0] + 1 if do_backtrack else k
                    if not do_backtrack and start < seen[0] + 1:
                        continue
                    if start not in seen:
                        raise Abort("starting motion frame")
                    i0 = seen.index(start)
                    for i in range(i0, len(seen)):
                        fk, fk1 = seen[i], seen[i - 1]
                        if fk != fk1 + 1:
                            raise Abort("non-consecutive")
                        if fk > k:
                            break
                        Xk1 = self.sensor_pose(fk1)
                        if Xk1 is None:
                            raise Abort("cam pose query")
                        Xk = self.init_or_lin_pose(fk1)  # sic: the reference reads k-1 here
                        self._point_update(t, o, fk1, fk, Xk, Xk1, i == i0, affected, local)
                        for key, v in local["values"].items():
                            if key in self.theta:
                                raise Abort("ValuesKeyAlreadyExists")
                            self.theta[key] = v
                        local["values"] = {}
                else:
                    self._point_update(t, o, k - 1, k, self.init_or_lin_pose(k), self.init_or_lin_pose(k - 1),
                                       False, affected, local)
                    for key, v in local["values"].items():
                        if key in self.theta:
                            raise Abort("ValuesKeyAlreadyExists")
                        self.theta[key] = v
        for o in sorted(affected):
            frames = sorted(affected[o])
            if len(frames) < 2:
                raise Abort("affected frames < 2")
            for idx, f in enumerate(frames):
                self._object_update(f, o, idx > 0, out)
        self.factors.extend(out)


def noise_models(shipped=True, robust=True):
    hk = 1e-4 if robust else 0.0
    odo = [0.05] * 3 + [0.1] * 3 if shipped else [0.02] * 3 + [0.01] * 3
    sm = [0.01] * 3 + ([0.01] * 3 if shipped else [0.1] * 3)
    return dict(static=([0.06] * 3, hk), dynamic=([0.0625] * 3, hk),
                motion=([1e-5 if shipped else 0.01] * 3, hk), odometry=(odo, 0.0), smoothing=(sm, 0.0),
                prior=([1e-4] * 6, 0.0))


class SlidingWindow:
    def __init__(self, window, overlap):
        self.window, self.overlap, self.prev, self.first = window, overlap, overlap, -1

    def check(self, k):
        if self.first == -1:
            self.first = k
        frame = k - self.first
        cond = (self.prev - (frame - self.window)) == self.overlap
        if cond:
            self.prev = frame
        return cond, k - self.window, k


def add_packet(mp, pk):
    for arr in (pk.static_measurements, pk.dynamic_measurements):
        for r in arr:
            mp.add(int(r["tracklet_id"]), int(r["object_id"]), int(r["frame_id"]), r["landmark"])
    mp.frames[pk.frame_id]["X"] = np.asarray(pk.T_world_camera, float)
    mp.frames[pk.frame_id]["motions"] = {int(o): np.asarray(v, float) for o, v in pk.estimated_motions.items()}


def construct_graph(mp, frm, to, kw):
    u = Formulation(mp, **kw)
    for f in range(frm, to + 1):
        T = mp.frames[f]["X"]
        if f == frm:
            u.set_initial_pose(f, T)
            u.set_initial_pose_prior(f, T)
        else:
            u.add_odometry(f, T)
            u.update_dynamic(f)
        u.update_static(f)
    return u


def run_stream(packets, full_batch=True, window=10, overlap=4, **kw):
    """Feeds the packets through the restated spin; returns (main
    formulation, [window formulations built by constructGraph])."""
    mp = Map()
    main = Formulation(mp, **kw)
    sw = SlidingWindow(window, overlap)
    windows = []
    for i, pk in enumerate(packets):
        add_packet(mp, pk)
        k = pk.frame_id
        if i == 0:
            sw.check(k)
            main.set_initial_pose(k, pk.T_world_camera)
            main.set_initial_pose_prior(k, pk.T_world_camera)
            continue
        main.add_odometry(k, pk.T_world_camera)
        main.update_static(k)
        main.update_dynamic(k)
        if not full_batch:
            cond, s, e = sw.check(k)
            if cond:
                windows.append((s, e, construct_graph(mp, s, e, kw)))
    return main, windows


def eigen_quaternion(R):
    """Eigen::Quaternion(Matrix3) (quaternionbase_assign_impl), as
    gtsam::Rot3::toQuaternion returns it; (x, y, z, w)."""
    m = np.asarray(R, float).reshape(3, 3)
    t = m[0, 0] + m[1, 1] + m[2, 2]
    if t > 0.0:
        t = np.sqrt(t + 1.0)
        w = 0.5 * t
        t = 0.5 / t
        return ((m[2, 1] - m[1, 2]) * t, (m[0, 2] - m[2, 0]) * t, (m[1, 0] - m[0, 1]) * t, w)
    i = 0
    if m[1, 1] > m[0, 0]:
        i = 1
    if m[2, 2] > m[i, i]:
        i = 2
    j, k = (i + 1) % 3, (i + 2) % 3
    c = [0.0, 0.0, 0.0]
    t = np.sqrt(m[i, i] - m[j, j] - m[k, k] + 1.0)
    c[i] = 0.5 * t
    t = 0.5 / t
    w = (m[k, j] - m[j, k]) * t
    c[j] = (m[j, i] + m[i, j]) * t
    c[k] = (m[k, i] + m[i, k]) * t
    return (c[0], c[1], c[2], w)


def csv_field(v):
    """One value streamed into a default-formatted std::stringstream
    (CsvWriter::add, utils/CsvParser.hpp:279-289)."""
    if isinstance(v, (int, np.integer)):
        return str(int(v))
    return "%g" % float(v)


def pose_fields(p12, gt12):
    q, g = eigen_quaternion(p12[:9]), eigen_quaternion(gt12[:9])
    return list(p12[9:12]) + list(q) + list(gt12[9:12]) + list(g)
