// synth.cpp — deterministic synthetic backend graphs (see include/dynosynth.h).
//
// Structure follows the reference WorldMotion / WorldPose formulations with
// do_backtrack = false (Formulation-impl.hpp:203-584,
// WorldMotionEstimator.cc:155-316, WorldPoseEstimator.cc:84-286); sizes and
// noise follow SURVEY.md §8(d) and dynosam/params/backend.flags:8-48.
#include "../../include/dynosynth.h"

#include <cmath>
#include <cstring>
#include <random>
#include <vector>

namespace {

struct Pose {
  double R[9];
  double t[3];
};

Pose identity() {
  Pose p;
  std::memset(&p, 0, sizeof(p));
  p.R[0] = p.R[4] = p.R[8] = 1.0;
  return p;
}

Pose compose(const Pose& a, const Pose& b) {
  Pose c;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j)
      c.R[3 * i + j] = a.R[3 * i] * b.R[j] + a.R[3 * i + 1] * b.R[3 + j] + a.R[3 * i + 2] * b.R[6 + j];
    c.t[i] = a.R[3 * i] * b.t[0] + a.R[3 * i + 1] * b.t[1] + a.R[3 * i + 2] * b.t[2] + a.t[i];
  }
  return c;
}

Pose inverse(const Pose& a) {
  Pose c;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) c.R[3 * i + j] = a.R[3 * j + i];
  for (int i = 0; i < 3; ++i)
    c.t[i] = -(c.R[3 * i] * a.t[0] + c.R[3 * i + 1] * a.t[1] + c.R[3 * i + 2] * a.t[2]);
  return c;
}

void transform_from(const Pose& T, const double* p, double* o) {
  for (int i = 0; i < 3; ++i) o[i] = T.R[3 * i] * p[0] + T.R[3 * i + 1] * p[1] + T.R[3 * i + 2] * p[2] + T.t[i];
}

void transform_to(const Pose& T, const double* p, double* o) {
  const double d[3] = {p[0] - T.t[0], p[1] - T.t[1], p[2] - T.t[2]};
  for (int i = 0; i < 3; ++i) o[i] = T.R[i] * d[0] + T.R[3 + i] * d[1] + T.R[6 + i] * d[2];
}

// SE(3) exponential, tangent [w; v] (GTSAM Pose3::Expmap convention)
Pose expmap(const double* xi) {
  const double* w = xi;
  const double* v = xi + 3;
  const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  Pose T = identity();
  const double W[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
  if (th2 <= 2.220446049250313e-16) {
    for (int i = 0; i < 9; ++i) T.R[i] += W[i];
    for (int i = 0; i < 3; ++i) T.t[i] = v[i];
    return T;
  }
  const double th = std::sqrt(th2);
  double K[9], KK[9];
  for (int i = 0; i < 9; ++i) K[i] = W[i] / th;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) KK[3 * i + j] = K[3 * i] * K[j] + K[3 * i + 1] * K[3 + j] + K[3 * i + 2] * K[6 + j];
  const double s = std::sin(th), s2 = std::sin(th / 2.0), omc = 2.0 * s2 * s2;
  for (int i = 0; i < 9; ++i) T.R[i] += s * K[i] + omc * KK[i];
  const double wv = w[0] * v[0] + w[1] * v[1] + w[2] * v[2];
  const double wxv[3] = {w[1] * v[2] - w[2] * v[1], w[2] * v[0] - w[0] * v[2], w[0] * v[1] - w[1] * v[0]};
  double Rwxv[3];
  for (int i = 0; i < 3; ++i) Rwxv[i] = T.R[3 * i] * wxv[0] + T.R[3 * i + 1] * wxv[1] + T.R[3 * i + 2] * wxv[2];
  for (int i = 0; i < 3; ++i) T.t[i] = (wxv[i] - Rwxv[i] + w[i] * wv) / th2;
  return T;
}

class Rng {
 public:
  explicit Rng(uint64_t seed) : gen_(seed) {}
  double uniform() { return static_cast<double>(gen_() >> 11) * (1.0 / 9007199254740992.0); }
  // Box–Muller, one value per call (no caching: deterministic order)
  double normal(double sigma) {
    const double u1 = 1.0 - uniform();  // (0, 1]
    const double u2 = uniform();
    return sigma * std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
  }
  int uniform_int(int lo, int hi) {  // inclusive
    if (hi <= lo) return lo;
    return lo + static_cast<int>(gen_() % static_cast<uint64_t>(hi - lo + 1));
  }

 private:
  std::mt19937_64 gen_;
};

uint64_t symbol(unsigned char c, uint64_t j) { return (static_cast<uint64_t>(c) << 56) | (j & ((1ULL << 56) - 1)); }
uint64_t labeled(unsigned char c, unsigned char l, uint64_t j) {
  return (static_cast<uint64_t>(c) << 56) | (static_cast<uint64_t>(l) << 48) | (j & ((1ULL << 48) - 1));
}
uint64_t cantor(uint64_t a, uint64_t b) { return ((a + b) * (a + b + 1) / 2) + b; }

struct Block {
  std::vector<uint64_t> keys;
  std::vector<double> meas, sigmas, huber;
  size_t n = 0;
};

void put_pose(std::vector<double>& v, const Pose& p) {
  v.insert(v.end(), p.R, p.R + 9);
  v.insert(v.end(), p.t, p.t + 3);
}

}  // namespace

struct dynosynth {
  Block b[6];
  std::vector<uint64_t> vkeys;
  std::vector<uint8_t> vkinds;
  std::vector<double> vdata, gt;
};

extern "C" {

void dynosynth_config_default(dynosynth_config* c) {
  c->frames = 50;
  c->objects = 1;
  c->static_landmarks = 1460;
  c->dyn_slots = 12;
  c->static_track_len = 8;
  c->dyn_track_len = 10;
  c->seed = 42;
  c->noise_code_defaults = 0;
  c->object_visible_frames = 0;
  c->formulation = 0;
  c->smoothing = 1;
  c->robust = 1;
}

int dynosynth_generate(const dynosynth_config* c, dynosynth** out) {
  *out = nullptr;
  if (!c || c->frames < 2 || c->objects < 0 || c->static_landmarks < 0 || c->dyn_slots < 0 ||
      c->static_track_len < 2 || c->dyn_track_len < 3 || c->objects > 200)
    return DYNOHIP_EINVAL;
  dynosynth* s = new dynosynth();
  Rng rng(c->seed);
  const int F = c->frames;
  // noise (backend.flags:8-24 or BackendParams.cc:26-40)
  double odo_r = 0.05, odo_t = 0.1, sm_r = 0.01, sm_t = 0.01, tern = 1e-5;
  if (c->noise_code_defaults) { odo_r = 0.02; odo_t = 0.01; sm_r = 0.01; sm_t = 0.1; tern = 0.01; }
  const double st_sigma = 0.06, dyn_sigma = 0.0625, huber = c->robust ? 1e-4 : 0.0, prior_sigma = 1e-4;
  const double meas_noise = 0.01;

  auto add_value_pose = [&](uint64_t key, const Pose& init, const Pose& truth) {
    s->vkeys.push_back(key);
    s->vkinds.push_back(DYNOHIP_POSE3);
    put_pose(s->vdata, init);
    put_pose(s->gt, truth);
  };
  auto add_value_point = [&](uint64_t key, const double* init, const double* truth) {
    s->vkeys.push_back(key);
    s->vkinds.push_back(DYNOHIP_POINT3);
    s->vdata.insert(s->vdata.end(), init, init + 3);
    s->gt.insert(s->gt.end(), truth, truth + 3);
  };
  auto add_factor = [&](int t, std::initializer_list<uint64_t> keys, const double* meas, int mdim,
                        std::initializer_list<double> sig, double k) {
    Block& B = s->b[t];
    B.keys.insert(B.keys.end(), keys);
    if (mdim) B.meas.insert(B.meas.end(), meas, meas + mdim);
    B.sigmas.insert(B.sigmas.end(), sig);
    B.huber.push_back(k);
    B.n++;
  };

  // camera: ground truth with constant twist; frontend = random walk
  const double xi_c[6] = {0.01, 0.02, 0.005, 0.5, 0.0, 0.05};
  const Pose step_c = expmap(xi_c);
  std::vector<Pose> X(F), Xfe(F);
  X[0] = identity();
  Xfe[0] = identity();
  for (int k = 1; k < F; ++k) {
    X[k] = compose(X[k - 1], step_c);
    double n[6];
    for (int i = 0; i < 3; ++i) n[i] = rng.normal(0.005);
    for (int i = 3; i < 6; ++i) n[i] = rng.normal(0.02);
    Xfe[k] = compose(compose(Xfe[k - 1], step_c), expmap(n));
  }
  for (int k = 0; k < F; ++k) add_value_pose(symbol('X', k), Xfe[k], X[k]);
  {
    double m[12];
    std::memcpy(m, Xfe[0].R, sizeof(Xfe[0].R));
    std::memcpy(m + 9, Xfe[0].t, sizeof(Xfe[0].t));
    add_factor(3, {symbol('X', 0)}, m, 12, {prior_sigma, prior_sigma, prior_sigma, prior_sigma, prior_sigma, prior_sigma}, 0.0);
  }
  for (int k = 1; k < F; ++k) {
    const Pose odom = compose(inverse(Xfe[k - 1]), Xfe[k]);
    double m[12];
    std::memcpy(m, odom.R, sizeof(odom.R));
    std::memcpy(m + 9, odom.t, sizeof(odom.t));
    add_factor(2, {symbol('X', k - 1), symbol('X', k)}, m, 12, {odo_r, odo_r, odo_r, odo_t, odo_t, odo_t}, 0.0);
  }

  // static landmarks
  const int Ls = std::min(c->static_track_len, F);
  for (int i = 0; i < c->static_landmarks; ++i) {
    const int s0 = rng.uniform_int(0, F - Ls);
    const Pose& Xm = X[s0 + Ls / 2];
    const double local[3] = {rng.normal(6.0), rng.normal(3.0), 12.0 + rng.normal(4.0)};
    double p[3];
    transform_from(Xm, local, p);
    const uint64_t key = symbol('l', static_cast<uint64_t>(i));
    double init[3] = {0, 0, 0};
    for (int k = s0; k < s0 + Ls; ++k) {
      double z[3];
      transform_to(X[k], p, z);
      for (int j = 0; j < 3; ++j) z[j] += rng.normal(meas_noise);
      if (k == s0) continue;  // first observation dropped (no backtrack)
      if (k == s0 + 1) transform_from(Xfe[k], z, init);
      add_factor(0, {symbol('X', k), key}, z, 3, {st_sigma, st_sigma, st_sigma}, huber);
    }
    add_value_point(key, init, p);
  }

  // dynamic objects
  const int Ld = c->dyn_track_len;
  uint64_t next_tracklet = static_cast<uint64_t>(c->static_landmarks);
  for (int j = 0; j < c->objects; ++j) {
    const unsigned char label = static_cast<unsigned char>('0' + j + 1);
    int v0 = 0, v1 = F - 1;
    if (c->object_visible_frames > 0 && c->object_visible_frames < F) {
      v0 = rng.uniform_int(0, F - c->object_visible_frames);
      v1 = v0 + c->object_visible_frames - 1;
    }
    // ground-truth object poses: body-frame constant twist
    double xi_o[6];
    for (int i = 0; i < 3; ++i) xi_o[i] = rng.normal(0.02);
    xi_o[3] = 0.5 + rng.normal(0.3);
    xi_o[4] = rng.normal(0.3);
    xi_o[5] = rng.normal(0.3);
    const Pose step_o = expmap(xi_o);
    std::vector<Pose> L(F);
    {
      Pose L0 = identity();
      L0.t[0] = rng.normal(3.0);
      L0.t[1] = rng.normal(1.0);
      L0.t[2] = 8.0 + rng.normal(2.0);
      L[0] = compose(X[0], L0);
      for (int k = 1; k < F; ++k) L[k] = compose(L[k - 1], step_o);
    }
    std::vector<int> motion_used(F, 0), pose_used(F, 0);
    for (int q = 0; q < c->dyn_slots; ++q) {
      for (int a = v0 + (q * Ld) / std::max(1, c->dyn_slots); a + Ld - 1 <= v1; a += Ld) {
        const uint64_t trk = next_tracklet++;
        const double body[3] = {rng.normal(1.0), rng.normal(1.0), rng.normal(1.0)};
        std::vector<double> z(3 * Ld), pw(3 * Ld);
        for (int k = a; k < a + Ld; ++k) {
          transform_from(L[k], body, &pw[3 * (k - a)]);
          transform_to(X[k], &pw[3 * (k - a)], &z[3 * (k - a)]);
          for (int d = 0; d < 3; ++d) z[3 * (k - a) + d] += rng.normal(meas_noise);
        }
        // points from the second observation on (first one dropped)
        for (int k = a + 1; k < a + Ld; ++k) {
          const uint64_t key = symbol('m', cantor(trk, static_cast<uint64_t>(k)));
          double init[3];
          transform_from(Xfe[k], &z[3 * (k - a)], init);
          add_value_point(key, init, &pw[3 * (k - a)]);
          add_factor(0, {symbol('X', k), key}, &z[3 * (k - a)], 3, {dyn_sigma, dyn_sigma, dyn_sigma}, huber);
          if (k >= a + 2) {
            const uint64_t kprev = symbol('m', cantor(trk, static_cast<uint64_t>(k - 1)));
            if (c->formulation == 0) {
              add_factor(1, {kprev, key, labeled('H', label, static_cast<uint64_t>(k))}, nullptr, 0, {tern, tern, tern}, huber);
              motion_used[k] = 1;
            } else {
              add_factor(4, {kprev, key, labeled('L', label, static_cast<uint64_t>(k - 1)), labeled('L', label, static_cast<uint64_t>(k))},
                         nullptr, 0, {tern, tern, tern}, huber);
              pose_used[k] = pose_used[k - 1] = 1;
            }
          }
        }
      }
    }
    for (int k = 0; k < F; ++k) {
      if (c->formulation == 0 && motion_used[k]) {
        const Pose H = compose(L[k], inverse(L[k - 1]));
        add_value_pose(labeled('H', label, static_cast<uint64_t>(k)), identity(), H);
        if (c->smoothing && k >= 2 && motion_used[k - 1]) {
          double m[12];
          const Pose I = identity();
          std::memcpy(m, I.R, sizeof(I.R));
          std::memcpy(m + 9, I.t, sizeof(I.t));
          add_factor(2, {labeled('H', label, static_cast<uint64_t>(k - 1)), labeled('H', label, static_cast<uint64_t>(k))}, m, 12,
                     {sm_r, sm_r, sm_r, sm_t, sm_t, sm_t}, 0.0);
        }
      }
      if (c->formulation == 1 && pose_used[k]) {
        double n[6];
        for (int i = 0; i < 3; ++i) n[i] = rng.normal(0.02);
        for (int i = 3; i < 6; ++i) n[i] = rng.normal(0.1);
        add_value_pose(labeled('L', label, static_cast<uint64_t>(k)), compose(L[k], expmap(n)), L[k]);
        if (c->smoothing && k >= 2 && pose_used[k - 1] && pose_used[k - 2])
          add_factor(5, {labeled('L', label, static_cast<uint64_t>(k - 2)), labeled('L', label, static_cast<uint64_t>(k - 1)),
                         labeled('L', label, static_cast<uint64_t>(k))},
                     nullptr, 0, {sm_r, sm_r, sm_r, sm_t, sm_t, sm_t}, 0.0);
      }
    }
  }
  *out = s;
  return DYNOHIP_OK;
}

void dynosynth_destroy(dynosynth* s) { delete s; }

void dynosynth_graph(const dynosynth* s, dynohip_graph_view* g) {
  dynohip_factor_block* dst[6] = {&g->pose_to_point, &g->landmark_motion_ternary, &g->between,
                                  &g->prior, &g->landmark_motion_pose, &g->landmark_pose_smoothing};
  for (int t = 0; t < 6; ++t) {
    const Block& B = s->b[t];
    dst[t]->n = B.n;
    dst[t]->keys = B.keys.empty() ? nullptr : B.keys.data();
    dst[t]->measured = B.meas.empty() ? nullptr : B.meas.data();
    dst[t]->sigmas = B.sigmas.empty() ? nullptr : B.sigmas.data();
    dst[t]->huber_k = B.huber.empty() ? nullptr : B.huber.data();
  }
}
size_t dynosynth_num_values(const dynosynth* s) { return s->vkeys.size(); }
size_t dynosynth_values_len(const dynosynth* s) { return s->vdata.size(); }
const uint64_t* dynosynth_value_keys(const dynosynth* s) { return s->vkeys.data(); }
const uint8_t* dynosynth_value_kinds(const dynosynth* s) { return s->vkinds.data(); }
const double* dynosynth_value_data(const dynosynth* s) { return s->vdata.data(); }
const double* dynosynth_ground_truth(const dynosynth* s) { return s->gt.data(); }

}  // extern "C"
