"""Frontend-output replay reader (dynosam_amd/csrc/replay.cpp through
dynosam_amd.replay) — SURVEY.md §8(f) row 2.

The reference's replay file is nlohmann BSON of
std::map<FrameId, RGBDInstanceOutputPacket> (Logger.hpp:170-230,
JsonUtils.cc:64-118). No such file ships with the reference (the OMD
sequence is an external download), so the files here are written by the
restated encoder tests/bson_frontend.py: the reader is pinned against that
restatement, and "parity unpinned" against the reference's own files.
"""
import numpy as np
import pytest

from dynosam_amd import backend, stream
from dynosam_amd.backend import BackendError
from dynosam_amd.replay import FrontendReplay, load_frontend_output

import bson_frontend as bf

CFG = stream.StreamConfig(frames=24, objects=2, static_landmarks=120, dyn_slots=6)


def _gt(packets, gt):
    out = {}
    for pk in packets:
        k = pk.frame_id
        objs = {o: (stream.pose12(Ls[k]), stream.pose12(Ls[k] @ stream.inv(Ls[k - 1])) if k else None)
                for o, Ls in gt["L"].items()}
        out[k] = bf.gt_json(k, stream.pose12(gt["X"][k]), objs, timestamp=pk.timestamp)
    return out


def test_round_trip_packets(tmp_path):
    packets, gt = stream.generate(CFG)
    path = tmp_path / "rgbd_frontend_output.bson"
    bf.write_frontend_output(path, packets, _gt(packets, gt))
    rp = FrontendReplay(path)
    assert len(rp) == len(packets)
    for pk, got in zip(packets, rp.packets()):
        assert got.frame_id == pk.frame_id and got.timestamp == pk.timestamp
        for a, b in ((pk.static_measurements, got.static_measurements),
                     (pk.dynamic_measurements, got.dynamic_measurements)):
            for f in ("tracklet_id", "object_id", "frame_id", "landmark"):
                np.testing.assert_array_equal(a[f], b[f])  # doubles survive BSON exactly
        # Pose3 goes through a quaternion (JsonUtils.hpp:181-206)
        np.testing.assert_allclose(got.T_world_camera, pk.T_world_camera, rtol=0, atol=4e-15)
        assert sorted(got.estimated_motions) == sorted(pk.estimated_motions)
        for o in pk.estimated_motions:
            np.testing.assert_allclose(got.estimated_motions[o], pk.estimated_motions[o], rtol=0, atol=4e-15)
    X, objs = rp.ground_truth(5)
    np.testing.assert_allclose(X, stream.pose12(gt["X"][5]), atol=4e-15)
    assert sorted(objs) == sorted(gt["L"])
    assert rp.ground_truth(0)[1][1][1] is None  # prev_H_current_world absent at frame 0


def test_replayed_stream_builds_the_same_graph(tmp_path):
    packets, _ = stream.generate(CFG)
    path = tmp_path / "f.bson"
    bf.write_frontend_output(path, packets)
    graphs = []
    for pks in (packets, load_frontend_output(path)):
        m = backend.RGBDBackendModule(full_batch_frame=len(pks), optimize=False)
        for p in pks:
            m.spinOnce(p)
        graphs.append((m.formulation.getGraph(), m.formulation.getTheta()))
    (g0, v0), (g1, v1) = graphs
    for t in g0.arrays():
        a, b = g0.arrays()[t], g1.arrays()[t]
        np.testing.assert_array_equal(a[0], b[0])
        if a[1] is not None:
            tol = 0 if t == "pose_to_point" else 1e-14
            np.testing.assert_allclose(a[1], b[1], rtol=0, atol=tol)
    np.testing.assert_array_equal(v0.keys, v1.keys)
    np.testing.assert_allclose(v0.data, v1.data, rtol=0, atol=1e-12)


def test_integer_encodings():
    # int64 tracklet ids, frame ids beyond int32 (BSON 0x12), and a uint64 frame (0x11)
    pk = backend.RGBDInstanceOutputPacket(
        frame_id=2**33, T_world_camera=stream.pose12(np.eye(4)),
        static_measurements=backend.make_measurements([2**40], [0], [2**33], [[1.0, 2.0, 3.0]]),
        dynamic_measurements=backend.make_measurements([7], [3], [2**33], [[0.5, 0.25, 4.0]]),
        estimated_motions={3: stream.pose12(stream.expmap([0.1, 0.0, 0.0, 1.0, 0.0, 0.0]))})
    blob = bf.to_bson({"data": [[bf.U64(pk.frame_id), bf.packet_json(pk)]]})
    got = FrontendReplay(data=blob).packet(0)
    assert got.frame_id == 2**33
    assert int(got.static_measurements["tracklet_id"][0]) == 2**40
    assert int(got.dynamic_measurements["object_id"][0]) == 3
    np.testing.assert_allclose(got.estimated_motions[3], pk.estimated_motions[3], atol=4e-15)


def _one_packet_blob(mutate):
    packets, _ = stream.generate(stream.StreamConfig(frames=3, objects=1, static_landmarks=10, dyn_slots=3))
    j = bf.packet_json(packets[1])
    mutate(j)
    return bf.to_bson({"data": [[bf.U64(1), j]]})


@pytest.mark.parametrize("name,mutate", [
    ("keypoint list shorter", lambda j: j["static_keypoints"].pop()),
    ("tracklet mismatch", lambda j: j["static_keypoints"][0].__setitem__("tracklet_id", 999999)),
    ("landmark not LOCAL", lambda j: j["static_landmarks"][0].__setitem__("reference_frame", "global")),
    ("missing camera pose", lambda j: j.pop("T_world_camera")),
    ("map key differs", lambda j: j.__setitem__("frame_id", bf.U64(2))),
])
def test_malformed_packets_are_errors(name, mutate):
    with pytest.raises(BackendError):
        FrontendReplay(data=_one_packet_blob(mutate))


def test_truncated_and_unordered_files(tmp_path):
    packets, _ = stream.generate(stream.StreamConfig(frames=4, objects=1, static_landmarks=10, dyn_slots=3))
    blob = bf.to_bson({"data": [[bf.U64(p.frame_id), bf.packet_json(p)] for p in packets]})
    with pytest.raises(BackendError):
        FrontendReplay(data=blob[:-7])
    rev = bf.to_bson({"data": [[bf.U64(p.frame_id), bf.packet_json(p)] for p in packets[::-1]]})
    with pytest.raises(BackendError):
        FrontendReplay(data=rev)
    with pytest.raises(BackendError):
        FrontendReplay(tmp_path / "missing.bson")
