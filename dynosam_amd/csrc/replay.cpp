// replay.cpp — reader of the reference's frontend-output replay file
// (SURVEY.md §8(f) row 2): the BSON that RGBDInstanceFrontendModule writes
// with JsonConverter::WriteOutJson(std::map<FrameId, RGBDInstanceOutputPacket>)
// (dynosam/src/frontend/RGBDInstanceFrontendModule.cc:80,
//  dynosam/include/dynosam/logger/Logger.hpp:170-230) through
// nlohmann::json::to_bson. The JSON layout it decodes is the reference's:
//   {"data": [[frame_id, packet], ...]}   (std::map with a non-string key)
//   packet  JsonUtils.cc:68-118 (static/dynamic keypoints and landmarks,
//           T_world_camera, timestamp, frame_id, estimated_motions,
//           propogated_object_poses, camera_poses, ground_truth)
//   status  TrackedValueStatus<MeasurementWithCovariance<T>>
//           {value: {measurement: Eigen rows, covariance?}, frame_id,
//            tracklet_id, object_id, reference_frame}  (JsonUtils.hpp:289-343)
//   Pose3   {tx, ty, tz, qx, qy, qz, qw}               (JsonUtils.hpp:178-207)
//   ground truth  GroundTruthPacket.cc:296-353
// The backend reads, per packet, what RGBDBackendModule::updateMap reads
// (RGBDBackendModule.cc:266-278): the static and dynamic landmark+keypoint
// pairs (collectLandmarkKeypointMeasurementsHelper checks, with CHECKs, that
// the two lists agree element by element and that landmarks are LOCAL,
// RGBDInstance-Definitions.cc:42-66), the frontend camera pose and the
// estimated motions. Zero-copy: the reader walks the BSON in place.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/dynobackend.h"

namespace {

struct Err : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// BSON element types written by nlohmann::json::to_bson
enum : uint8_t {
  kDouble = 0x01, kString = 0x02, kDoc = 0x03, kArray = 0x04, kBinary = 0x05, kBool = 0x08, kNull = 0x0A,
  kInt32 = 0x10, kUInt64 = 0x11, kInt64 = 0x12
};

struct Val {
  uint8_t type = 0;
  const uint8_t* p = nullptr;  // value bytes
};

int32_t rd32(const uint8_t* p) {
  int32_t v;
  std::memcpy(&v, p, 4);
  return v;
}

// size in bytes of a value of `type` at p (bounded by end)
size_t value_size(uint8_t type, const uint8_t* p, const uint8_t* end) {
  auto need = [&](size_t n) {
    if (static_cast<size_t>(end - p) < n) throw Err("BSON: truncated value");
  };
  switch (type) {
    case kDouble: case kUInt64: case kInt64: need(8); return 8;
    case kInt32: need(4); return 4;
    case kBool: need(1); return 1;
    case kNull: return 0;
    case kString: { need(4); const int32_t n = rd32(p); if (n < 1) throw Err("BSON: bad string"); need(4 + static_cast<size_t>(n)); return 4 + n; }
    case kDoc: case kArray: { need(4); const int32_t n = rd32(p); if (n < 5) throw Err("BSON: bad document"); need(static_cast<size_t>(n)); return n; }
    case kBinary: { need(5); const int32_t n = rd32(p); if (n < 0) throw Err("BSON: bad binary"); need(5 + static_cast<size_t>(n)); return 5 + n; }
    default: throw Err("BSON: unsupported element type " + std::to_string(type));
  }
}

// iterate the elements of a document / array value; fn returns false to stop
template <typename Fn>
void each(const Val& v, Fn&& fn) {
  if (v.type != kDoc && v.type != kArray) throw Err("BSON: not a document");
  const int32_t n = rd32(v.p);
  const uint8_t* q = v.p + 4;
  const uint8_t* dend = v.p + n - 1;  // trailing 0x00
  if (*dend != 0) throw Err("BSON: document not terminated");
  while (q < dend) {
    const uint8_t t = *q++;
    const char* name = reinterpret_cast<const char*>(q);
    const void* z = std::memchr(q, 0, dend - q);
    if (!z) throw Err("BSON: unterminated element name");
    q = static_cast<const uint8_t*>(z) + 1;
    const size_t sz = value_size(t, q, dend);
    if (!fn(name, Val{t, q})) return;
    q += sz;
  }
}

Val field(const Val& doc, const char* key, bool required = true) {
  Val out;
  each(doc, [&](const char* name, const Val& e) {
    if (std::strcmp(name, key) == 0) {
      out = e;
      return false;
    }
    return true;
  });
  if (required && out.type == 0) throw Err(std::string("BSON: missing field '") + key + "'");
  return out;
}

std::vector<Val> items(const Val& arr) {
  std::vector<Val> out;
  each(arr, [&](const char*, const Val& e) {
    out.push_back(e);
    return true;
  });
  return out;
}

double num(const Val& v) {
  switch (v.type) {
    case kDouble: { double d; std::memcpy(&d, v.p, 8); return d; }
    case kInt32: return rd32(v.p);
    case kInt64: { int64_t i; std::memcpy(&i, v.p, 8); return static_cast<double>(i); }
    case kUInt64: { uint64_t u; std::memcpy(&u, v.p, 8); return static_cast<double>(u); }
    default: throw Err("BSON: not a number");
  }
}
int64_t integer(const Val& v) {
  switch (v.type) {
    case kInt32: return rd32(v.p);
    case kInt64: case kUInt64: { int64_t i; std::memcpy(&i, v.p, 8); return i; }
    default: throw Err("BSON: not an integer");
  }
}
std::string str(const Val& v) {
  if (v.type != kString) throw Err("BSON: not a string");
  return std::string(reinterpret_cast<const char*>(v.p + 4), rd32(v.p) - 1);
}

// gtsam::Pose3 from {tx..qw}: Rot3(qw, qx, qy, qz) is Eigen's
// Quaternion::toRotationMatrix (no normalisation), JsonUtils.hpp:195-206
void pose(const Val& v, double* out12) {
  const double w = num(field(v, "qw")), x = num(field(v, "qx")), y = num(field(v, "qy")), z = num(field(v, "qz"));
  const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
  const double twx = tx * w, twy = ty * w, twz = tz * w;
  const double txx = tx * x, txy = ty * x, txz = tz * x;
  const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
  const double R[9] = {1 - (tyy + tzz), txy - twz, txz + twy, txy + twz, 1 - (txx + tzz), tyz - twx,
                       txz - twy, tyz + twx, 1 - (txx + tyy)};
  std::memcpy(out12, R, sizeof(R));
  out12[9] = num(field(v, "tx"));
  out12[10] = num(field(v, "ty"));
  out12[11] = num(field(v, "tz"));
}

// Eigen column vector: [[a], [b], ...] (JsonUtils.hpp:155-176)
void eigen_vec(const Val& v, double* out, int n) {
  const auto rows = items(v);
  if (static_cast<int>(rows.size()) != n) throw Err("BSON: vector has the wrong size");
  for (int r = 0; r < n; ++r) {
    const auto c = items(rows[r]);
    if (c.size() != 1) throw Err("BSON: vector row is not 1 wide");
    out[r] = num(c[0]);
  }
}

struct Status {
  int64_t tracklet;
  int32_t object;
  uint64_t frame;
  std::string rf;
};
Status status(const Val& s) {
  Status o;
  o.tracklet = integer(field(s, "tracklet_id"));
  o.object = static_cast<int32_t>(integer(field(s, "object_id")));
  o.frame = static_cast<uint64_t>(integer(field(s, "frame_id")));
  o.rf = str(field(s, "reference_frame"));
  return o;
}

struct GtObject {
  int32_t object_id;
  double L_world[12];
  double prev_H[12];
  bool has_H;
};

struct Packet {
  uint64_t frame_id = 0;
  double timestamp = 0;
  double T_world_camera[12];
  std::vector<dynob_measurement> st, dy;
  std::vector<int32_t> motion_ids;
  std::vector<double> motions;
  bool has_gt = false;
  double gt_X[12];
  std::vector<GtObject> gt_objects;
};

// collectLandmarkKeypointMeasurementsHelper (RGBDInstance-Definitions.cc:42-66)
std::vector<dynob_measurement> landmark_keypoints(const Val& landmarks, const Val& keypoints) {
  const auto L = items(landmarks), K = items(keypoints);
  if (L.size() != K.size()) throw Err("landmark / keypoint lists differ in length");
  std::vector<dynob_measurement> out(L.size());
  for (size_t i = 0; i < L.size(); ++i) {
    const Status a = status(L[i]), b = status(K[i]);
    if (a.tracklet != b.tracklet || a.object != b.object || a.frame != b.frame)
      throw Err("landmark / keypoint status mismatch at index " + std::to_string(i));
    if (a.rf != "local") throw Err("backend landmarks must be in the LOCAL frame");
    dynob_measurement& m = out[i];
    std::memset(&m, 0, sizeof(m));
    m.tracklet_id = a.tracklet;
    m.object_id = a.object;
    m.frame_id = a.frame;
    eigen_vec(field(field(L[i], "value"), "measurement"), m.landmark, 3);
  }
  return out;
}

Packet packet(const Val& v) {
  Packet p;
  p.frame_id = static_cast<uint64_t>(integer(field(v, "frame_id")));
  p.timestamp = num(field(v, "timestamp"));
  pose(field(v, "T_world_camera"), p.T_world_camera);
  p.st = landmark_keypoints(field(v, "static_landmarks"), field(v, "static_keypoints"));
  p.dy = landmark_keypoints(field(v, "dynamic_landmarks"), field(v, "dynamic_keypoints"));
  // estimated_motions: std::map<ObjectId, ReferenceFrameValue<Motion3>> ->
  // [[object_id, {estimate, reference_frame}], ...]
  const Val em = field(v, "estimated_motions");
  if (em.type != kNull)
    for (const Val& kv : items(em)) {
      const auto pr = items(kv);
      if (pr.size() != 2) throw Err("estimated_motions entry is not a pair");
      p.motion_ids.push_back(static_cast<int32_t>(integer(pr[0])));
      double m[12];
      pose(field(pr[1], "estimate"), m);
      p.motions.insert(p.motions.end(), m, m + 12);
    }
  const Val gt = field(v, "ground_truth", false);
  if (gt.type == kDoc) {
    p.has_gt = true;
    pose(field(gt, "X_world"), p.gt_X);
    for (const Val& o : items(field(gt, "objects"))) {
      GtObject g{};
      g.object_id = static_cast<int32_t>(integer(field(o, "object_id")));
      pose(field(o, "L_world"), g.L_world);
      const Val h = field(o, "prev_H_current_world", false);
      g.has_H = h.type == kDoc;
      if (g.has_H) pose(h, g.prev_H);
      p.gt_objects.push_back(g);
    }
  }
  return p;
}

}  // namespace

struct dynob_replay {
  std::vector<uint8_t> bytes;
  std::vector<Packet> packets;
  std::string err;
};

extern "C" {

int dynob_replay_parse(const uint8_t* data, size_t n, dynob_replay** out) {
  if (!out || (!data && n)) return DYNOHIP_EINVAL;
  auto* r = new dynob_replay();
  *out = r;
  try {
    r->bytes.assign(data, data + n);
    if (n < 5 || rd32(r->bytes.data()) != static_cast<int32_t>(n) || r->bytes.back() != 0)
      throw Err("not a BSON document (size prefix / terminator)");
    const Val root{kDoc, r->bytes.data()};
    // std::map<FrameId, RGBDInstanceOutputPacket>: [[frame_id, packet], ...]
    for (const Val& kv : items(field(root, "data"))) {
      const auto pr = items(kv);
      if (pr.size() != 2) throw Err("data entry is not a [frame_id, packet] pair");
      Packet p = packet(pr[1]);
      if (static_cast<uint64_t>(integer(pr[0])) != p.frame_id) throw Err("map key differs from the packet frame id");
      r->packets.push_back(std::move(p));
    }
    for (size_t i = 1; i < r->packets.size(); ++i)
      if (r->packets[i].frame_id <= r->packets[i - 1].frame_id) throw Err("packets not in ascending frame order");
    return DYNOHIP_OK;
  } catch (const std::exception& e) {
    r->err = e.what();
    r->packets.clear();
    return DYNOHIP_EINVAL;
  }
}

int dynob_replay_open(const char* path, dynob_replay** out) {
  if (!path || !out) return DYNOHIP_EINVAL;
  std::ifstream f(path, std::ios::binary);
  if (!f.is_open()) {
    *out = new dynob_replay();
    (*out)->err = std::string("cannot open ") + path;
    return DYNOHIP_EINVAL;
  }
  const std::vector<uint8_t> b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  return dynob_replay_parse(b.data(), b.size(), out);
}

void dynob_replay_destroy(dynob_replay* r) { delete r; }
const char* dynob_replay_last_error(const dynob_replay* r) { return r ? r->err.c_str() : "null replay"; }
size_t dynob_replay_num_packets(const dynob_replay* r) { return r ? r->packets.size() : 0; }

int dynob_replay_packet(const dynob_replay* r, size_t i, dynob_input_packet* out) {
  if (!r || !out || i >= r->packets.size()) return DYNOHIP_EINVAL;
  const Packet& p = r->packets[i];
  std::memset(out, 0, sizeof(*out));
  out->frame_id = p.frame_id;
  out->timestamp = p.timestamp;
  std::memcpy(out->T_world_camera, p.T_world_camera, sizeof(p.T_world_camera));
  out->static_measurements = p.st.empty() ? nullptr : p.st.data();
  out->n_static = p.st.size();
  out->dynamic_measurements = p.dy.empty() ? nullptr : p.dy.data();
  out->n_dynamic = p.dy.size();
  out->motion_object_ids = p.motion_ids.empty() ? nullptr : p.motion_ids.data();
  out->motions12 = p.motions.empty() ? nullptr : p.motions.data();
  out->n_motions = p.motion_ids.size();
  return DYNOHIP_OK;
}

int dynob_replay_ground_truth(const dynob_replay* r, size_t i, double* X_world12, int32_t* object_ids,
                              double* L_world12, double* prev_H12, size_t cap, size_t* n_objects) {
  if (!r || i >= r->packets.size()) return DYNOHIP_EINVAL;
  const Packet& p = r->packets[i];
  if (n_objects) *n_objects = p.has_gt ? p.gt_objects.size() : 0;
  if (!p.has_gt) return 0;
  if (X_world12) std::memcpy(X_world12, p.gt_X, sizeof(p.gt_X));
  for (size_t k = 0; k < p.gt_objects.size() && k < cap; ++k) {
    const GtObject& g = p.gt_objects[k];
    if (object_ids) object_ids[k] = g.object_id;
    if (L_world12) std::memcpy(L_world12 + 12 * k, g.L_world, sizeof(g.L_world));
    if (prev_H12) {
      if (g.has_H)
        std::memcpy(prev_H12 + 12 * k, g.prev_H, sizeof(g.prev_H));
      else
        for (int j = 0; j < 12; ++j) prev_H12[12 * k + j] = std::nan("");
    }
  }
  return 1;
}

}  // extern "C"
