"""Fixture from the reference's exact-input test graph
(dynosam/test/test_rgbd_backend.cc:272-486, TEST(RGBDBackendModule,
testCliques)): 3 camera poses, 1 static landmark seen from all of them,
3 dynamic tracklets over frames 0-2 with 2 object motions, odometry
Betweens and a prior; Isotropic noise, no robust kernel.

Writes
  cliques.graph    the graph + initial values in the reference graph-file
                   format (dynosam_amd/graphio.py, round-trip precision);
  lm_cliques.json  the oracle's GTSAM-4.2 LM run on it (per-iteration
                   trace, final values by key). The oracle is not GTSAM:
                   this pins the restatement and the GPU path to each other
                   (LM outputs are parity-unpinned upstream).
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from dynosam_amd import graphio  # noqa: E402
from dynosam_amd.graph import NonlinearFactorGraph, Values  # noqa: E402
from dynosam_amd.keys import camera_pose_key as X, dynamic_landmark_key as M  # noqa: E402
from dynosam_amd.keys import object_motion_key as H, static_landmark_key as l  # noqa: E402


def expmap(w):
    w = np.asarray(w, dtype=np.float64)
    th = np.linalg.norm(w)
    K = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
    if th < 1e-12:
        return np.eye(3) + K
    return np.eye(3) + np.sin(th) / th * K + (1 - np.cos(th)) / th ** 2 * K @ K


class Pose:
    def __init__(self, R, t):
        self.R, self.t = np.asarray(R, dtype=np.float64), np.asarray(t, dtype=np.float64)

    def __mul__(self, o):
        if isinstance(o, Pose):
            return Pose(self.R @ o.R, self.R @ o.t + self.t)
        return self.R @ np.asarray(o, dtype=np.float64) + self.t

    def inverse(self):
        return Pose(self.R.T, -self.R.T @ self.t)

    def between(self, o):
        return self.inverse() * o

    def a12(self):
        return np.concatenate([self.R.reshape(9), self.t])


def build():
    H01 = Pose(expmap([0.3, 0.2, 0.1]), [0, 1, 1])       # Rot3::Rodrigues(0.3,0.2,0.1)
    H12 = Pose(expmap([0.5, 0.1, 0.1]), [1, 1.5, 1])
    H02 = H01 * H12
    dyn = [np.array([2, 1, 3.0]), np.array([1, 1, 3.0]), np.array([3, 0.5, 2.0])]
    pose = [Pose(expmap([0.2, 0.1, 0.12]), [1, 3, 4]), Pose(expmap([0.1, 0.2, 1.570796]), [1, 2, 1]),
            Pose(expmap([0.2, 0.3, 3.141593]), [2, 2, 1])]
    lm_sigma, pose_sigma = 10.0, 0.1
    g = NonlinearFactorGraph()
    for k, z in enumerate(([1, 2, 3], [2, 2, 3], [3, 2, 3])):
        g.add_pose_to_point(X(k), l(0), z, lm_sigma)
    for trk in (1, 2, 3):
        g.add_landmark_motion_ternary(M(0, trk), M(1, trk), H(1, 1), lm_sigma)
        g.add_landmark_motion_ternary(M(1, trk), M(2, trk), H(1, 2), lm_sigma)
    motions = [Pose(np.eye(3), np.zeros(3)), H01, H02]
    for trk in (1, 2, 3):
        for k in range(3):
            g.add_pose_to_point(X(k), M(k, trk), pose[k].inverse() * (motions[k] * dyn[trk - 1]), lm_sigma)
    g.add_between(X(0), X(1), pose[0].between(pose[1]).a12(), pose_sigma)
    g.add_between(X(1), X(2), pose[1].between(pose[2]).a12(), pose_sigma)
    g.add_prior(X(0), pose[0].a12(), pose_sigma)
    v = Values()
    v.insert_point(l(0), [0, 1, 1])
    for k in range(3):
        for trk in (1, 2, 3):
            v.insert_point(M(k, trk), motions[k] * dyn[trk - 1])
    v.insert_pose(H(1, 1), np.concatenate([np.eye(3).reshape(9), np.zeros(3)]))
    v.insert_pose(H(1, 2), np.concatenate([np.eye(3).reshape(9), np.zeros(3)]))
    for k in range(3):
        v.insert_pose(X(k), pose[k].a12())
    return g, v


def values_by_key(values, data):
    off = values._offsets()
    return {str(int(k)): [float(x) for x in data[off[i]:off[i + 1]]] for i, k in enumerate(values.keys)}


def main():
    from oracle_binding import Oracle
    g, v = build()
    path = os.path.join(HERE, "cliques.graph")
    graphio.write(path, g, v)
    g2, v2 = graphio.read(path)
    o = Oracle(g2, v2)
    s = o.optimize()
    out = {
        "source": "dynosam/test/test_rgbd_backend.cc:272-486 (testCliques), read back from cliques.graph",
        "iterations": s.iterations,
        "inner_iterations": s.inner_iterations,
        "initial_error": s.initial_error,
        "final_error": s.final_error,
        "trace": o.trace(),
        "final_values": values_by_key(v2, o.values_data()),
    }
    with open(os.path.join(HERE, "lm_cliques.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("iterations", s.iterations, "inner", s.inner_iterations, "error", s.initial_error, "->", s.final_error)


if __name__ == "__main__":
    main()
