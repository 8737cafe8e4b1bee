/*
 * oracle.c — CPU restatement of the DynoSAM backend hot path (see oracle.h).
 *
 * TEST INFRASTRUCTURE ONLY: the parity checker, never the product.
 * Plain C99, FP64, no external libraries. Single thread by default; with
 * oracle_set_threads(p, n > 1) the same LM runs its linearisation, errors
 * and Schur + envelope-Cholesky solve on n POSIX threads (the all-cores CPU
 * baseline of bench.py, SURVEY.md §8(d) "CPU baseline"): the same
 * operations, with the reductions split into fixed chunks and the envelope
 * Cholesky blocked right-looking, so results agree with the single-thread
 * path to rounding.
 */
#define _POSIX_C_SOURCE 200809L
#include "oracle.h"

#include <pthread.h>

#include <float.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* the shared transcendental functions (sin, tan, acos) of the pose
   arithmetic: the same IEEE operations as the kernels (se3.hpp), in place
   of glibc's, see trig.h. Built with -DORACLE_LIBM_TRIG (liboracle_libm.so)
   the oracle calls glibc's instead, as GTSAM does: the independent check
   that trig.h's rounding is not what makes the two sides agree
   (tests/test_trig.py, tests/test_gpu_parity.py). */
#ifdef ORACLE_LIBM_TRIG
#define dht_sin sin
#define dht_tan tan
#define dht_acos acos
#else
#include "../dynosam_amd/csrc/trig.h"
#endif

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* ------------------------------------------------------------------ */
/* 3x3 / SO(3) / SE(3) (GTSAM 4.2.0 Rot3 matrix rep, ROT3_EXPMAP,      */
/* POSE3_EXPMAP). Poses are 12 doubles: R row-major, t.                */
/* ------------------------------------------------------------------ */
static void m3_mul(const double* A, const double* B, double* C) {
  double T[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      T[3 * i + j] = A[3 * i + 0] * B[0 + j] + A[3 * i + 1] * B[3 + j] +
                     A[3 * i + 2] * B[6 + j];
  memcpy(C, T, sizeof(T));
}
static void m3_tr(const double* A, double* C) {
  double T[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) T[3 * i + j] = A[3 * j + i];
  memcpy(C, T, sizeof(T));
}
static void m3_mv(const double* A, const double* v, double* o) {
  double t[3];
  for (int i = 0; i < 3; ++i)
    t[i] = A[3 * i] * v[0] + A[3 * i + 1] * v[1] + A[3 * i + 2] * v[2];
  memcpy(o, t, sizeof(t));
}
static void m3_tmv(const double* A, const double* v, double* o) { /* A^T v */
  double t[3];
  for (int i = 0; i < 3; ++i)
    t[i] = A[i] * v[0] + A[3 + i] * v[1] + A[6 + i] * v[2];
  memcpy(o, t, sizeof(t));
}
static void skew(const double* w, double* W) {
  W[0] = 0.0;   W[1] = -w[2]; W[2] = w[1];
  W[3] = w[2];  W[4] = 0.0;   W[5] = -w[0];
  W[6] = -w[1]; W[7] = w[0];  W[8] = 0.0;
}
static void cross3(const double* a, const double* b, double* c) {
  double t[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2],
                 a[0] * b[1] - a[1] * b[0]};
  memcpy(c, t, sizeof(t));
}

/* so3::ExpmapFunctor (GTSAM 4.2.0 SO3.cpp) */
void oracle_rot_expmap(const double w[3], double R[9]) {
  const double theta2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  double W[9];
  skew(w, W);
  if (theta2 <= DBL_EPSILON) {
    for (int i = 0; i < 9; ++i) R[i] = W[i];
    R[0] += 1.0; R[4] += 1.0; R[8] += 1.0;
    return;
  }
  const double theta = sqrt(theta2);
  double K[9], KK[9];
  for (int i = 0; i < 9; ++i) K[i] = W[i] / theta;
  m3_mul(K, K, KK);
  const double s = dht_sin(theta);
  const double s2 = dht_sin(theta / 2.0);
  const double omc = 2.0 * s2 * s2;
  for (int i = 0; i < 9; ++i) R[i] = s * K[i] + omc * KK[i];
  R[0] += 1.0; R[4] += 1.0; R[8] += 1.0;
}

/* SO3::Logmap (GTSAM 4.2.0 SO3.cpp) */
void oracle_rot_logmap(const double R[9], double w[3]) {
  const double R11 = R[0], R12 = R[1], R13 = R[2];
  const double R21 = R[3], R22 = R[4], R23 = R[5];
  const double R31 = R[6], R32 = R[7], R33 = R[8];
  const double tr = R11 + R22 + R33;
  if (tr + 1.0 < 1e-3) {
    double W, Q1, Q2, Q3;
    int which;
    if (R33 > R22 && R33 > R11) {
      W = R21 - R12; Q1 = 2.0 + 2.0 * R33; Q2 = R31 + R13; Q3 = R23 + R32;
      which = 3;
    } else if (R22 > R11) {
      W = R13 - R31; Q1 = 2.0 + 2.0 * R22; Q2 = R23 + R32; Q3 = R12 + R21;
      which = 2;
    } else {
      W = R32 - R23; Q1 = 2.0 + 2.0 * R11; Q2 = R12 + R21; Q3 = R31 + R13;
      which = 1;
    }
    const double r = sqrt(Q1);
    const double one_over_r = 1 / r;
    const double norm = sqrt(Q1 * Q1 + Q2 * Q2 + Q3 * Q3 + W * W);
    const double sgn_w = W < 0 ? -1.0 : 1.0;
    const double mag = M_PI - (2 * sgn_w * W) / norm;
    const double scale = 0.5 * one_over_r * mag;
    if (which == 3) {
      w[0] = sgn_w * scale * Q2; w[1] = sgn_w * scale * Q3; w[2] = sgn_w * scale * Q1;
    } else if (which == 2) {
      w[0] = sgn_w * scale * Q3; w[1] = sgn_w * scale * Q1; w[2] = sgn_w * scale * Q2;
    } else {
      w[0] = sgn_w * scale * Q1; w[1] = sgn_w * scale * Q2; w[2] = sgn_w * scale * Q3;
    }
    return;
  }
  double magnitude;
  const double tr_3 = tr - 3.0;
  if (tr_3 < -1e-6) {
    const double theta = dht_acos((tr - 1.0) / 2.0);
    magnitude = theta / (2.0 * dht_sin(theta));
  } else {
    magnitude = 0.5 - tr_3 / 12.0 + tr_3 * tr_3 / 60.0;
  }
  w[0] = magnitude * (R32 - R23);
  w[1] = magnitude * (R13 - R31);
  w[2] = magnitude * (R21 - R12);
}

/* Pose3::Expmap (GTSAM 4.2.0 Pose3.cpp) */
void oracle_pose_expmap(const double xi[6], double T[12]) {
  const double* w = xi;
  const double* v = xi + 3;
  oracle_rot_expmap(w, T);
  const double theta2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  if (theta2 > DBL_EPSILON) {
    const double wv = w[0] * v[0] + w[1] * v[1] + w[2] * v[2];
    double tpar[3] = {w[0] * wv, w[1] * wv, w[2] * wv};
    double wxv[3], Rwxv[3];
    cross3(w, v, wxv);
    m3_mv(T, wxv, Rwxv);
    for (int i = 0; i < 3; ++i)
      T[9 + i] = (wxv[i] - Rwxv[i] + tpar[i]) / theta2;
  } else {
    T[9] = v[0]; T[10] = v[1]; T[11] = v[2];
  }
}

/* Pose3::Logmap (GTSAM 4.2.0 Pose3.cpp) */
void oracle_pose_logmap(const double T[12], double xi[6]) {
  double w[3];
  oracle_rot_logmap(T, w);
  const double* t = T + 9;
  const double th = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  xi[0] = w[0]; xi[1] = w[1]; xi[2] = w[2];
  if (th < 1e-10) {
    xi[3] = t[0]; xi[4] = t[1]; xi[5] = t[2];
    return;
  }
  double wn[3] = {w[0] / th, w[1] / th, w[2] / th};
  double W[9], WT[3], WWT[3];
  skew(wn, W);
  const double Tan = dht_tan(0.5 * th);
  m3_mv(W, t, WT);
  m3_mv(W, WT, WWT);
  const double c = 1 - th / (2. * Tan);
  for (int i = 0; i < 3; ++i) xi[3 + i] = t[i] - (0.5 * th) * WT[i] + c * WWT[i];
}

/* trig.h evaluated on n arguments: which 0 sin, 1 tan, 2 acos */
void oracle_trig(int which, const double* x, double* y, size_t n) {
  for (size_t i = 0; i < n; ++i)
    y[i] = which == 0 ? dht_sin(x[i]) : which == 1 ? dht_tan(x[i]) : dht_acos(x[i]);
}

void oracle_pose_compose(const double A[12], const double B[12], double C[12]) {
  double R[9], t[3];
  m3_mul(A, B, R);
  m3_mv(A, B + 9, t);
  for (int i = 0; i < 3; ++i) t[i] += A[9 + i];
  memcpy(C, R, sizeof(R));
  memcpy(C + 9, t, sizeof(t));
}

void oracle_pose_inverse(const double A[12], double C[12]) {
  double Rt[9], t[3];
  m3_tr(A, Rt);
  m3_mv(Rt, A + 9, t);
  memcpy(C, Rt, sizeof(Rt));
  C[9] = -t[0]; C[10] = -t[1]; C[11] = -t[2];
}

static void pose_transform_from(const double T[12], const double p[3], double o[3]) {
  double q[3];
  m3_mv(T, p, q);
  o[0] = q[0] + T[9]; o[1] = q[1] + T[10]; o[2] = q[2] + T[11];
}

/* Pose3::AdjointMap, tangent order [w; v]: [[R, 0], [t^ R, R]] */
static void pose_adjoint(const double T[12], double Ad[36]) {
  double tx[9], txR[9];
  skew(T + 9, tx);
  m3_mul(tx, T, txR);
  memset(Ad, 0, 36 * sizeof(double));
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      Ad[6 * i + j] = T[3 * i + j];
      Ad[6 * (i + 3) + j + 3] = T[3 * i + j];
      Ad[6 * (i + 3) + j] = txR[3 * i + j];
    }
}

static void pose_retract(const double T[12], const double xi[6], double o[12]) {
  double E[12];
  oracle_pose_expmap(xi, E);
  oracle_pose_compose(T, E, o);
}

/* ------------------------------------------------------------------ */
/* Keys                                                                */
/* ------------------------------------------------------------------ */
uint64_t oracle_cantor_pair(uint64_t k1, uint64_t k2) {
  return ((k1 + k2) * (k1 + k2 + 1) / 2) + k2;
}
void oracle_cantor_depair(uint64_t z, uint64_t* k1, uint64_t* k2) {
  uint64_t w = (uint64_t)floor(((sqrt((double)(z * 8 + 1))) - 1) / 2);
  uint64_t t = (w * (w + 1)) / 2;
  *k2 = z - t;
  *k1 = w - *k2;
}
uint64_t oracle_symbol(unsigned char c, uint64_t j) {
  return ((uint64_t)c << 56) | (j & ((1ULL << 56) - 1));
}
uint64_t oracle_labeled_symbol(unsigned char c, unsigned char label, uint64_t j) {
  return ((uint64_t)c << 56) | ((uint64_t)label << 48) | (j & ((1ULL << 48) - 1));
}
int oracle_reconstruct_labeled(uint64_t key, unsigned char expected_chr,
                               int* label, uint64_t* frame) {
  const unsigned char c = (unsigned char)(key >> 56);
  const unsigned char l = (unsigned char)((key >> 48) & 0xff);
  if (!(c > 0 && l > 0)) return 0;
  if (c != expected_chr) return 0;
  *frame = key & ((1ULL << 48) - 1);
  *label = (int)(char)l - '0';
  return 1;
}
unsigned char oracle_chr_extract(uint64_t key) {
  return (unsigned char)(key >> 56); /* same byte for Symbol and LabeledSymbol */
}

/* ------------------------------------------------------------------ */
/* Factors                                                             */
/* ------------------------------------------------------------------ */
enum { F_P2P = 0, F_TERN = 1, F_BTW = 2, F_PRIOR = 3, F_MP = 4, F_PS = 5, F_NT = 6 };
static const int kNKeys[F_NT] = {2, 3, 2, 1, 4, 3};
static const int kDim[F_NT] = {3, 3, 6, 6, 3, 6};
/* slot kinds: 0 = pose, 1 = point */
static const int kSlotKind[F_NT][4] = {
    {0, 1, -1, -1}, {1, 1, 0, -1}, {0, 0, -1, -1},
    {0, -1, -1, -1}, {1, 1, 0, 0}, {0, 0, 0, -1}};
static const int kMeasDim[F_NT] = {3, 0, 12, 12, 0, 0};

static int slot_dim(int type, int s) { return kSlotKind[type][s] == 0 ? 6 : 3; }
static int slot_vsize(int type, int s) { return kSlotKind[type][s] == 0 ? 12 : 3; }
int oracle_factor_dim(int type) { return (type >= 0 && type < F_NT) ? kDim[type] : -1; }
int oracle_factor_nkeys(int type) { return (type >= 0 && type < F_NT) ? kNKeys[type] : -1; }
int oracle_factor_cols(int type) {
  if (type < 0 || type >= F_NT) return -1;
  int c = 0;
  for (int s = 0; s < kNKeys[type]; ++s) c += slot_dim(type, s);
  return c;
}

/* residual only (used by all factors and by numerical derivatives) */
static void residual(int type, const double* const* v, const double* meas, double* r) {
  switch (type) {
    case F_P2P: { /* wTwi.transformTo(wPwp) - measured */
      const double* T = v[0];
      double d[3] = {v[1][0] - T[9], v[1][1] - T[10], v[1][2] - T[11]};
      double q[3];
      m3_tmv(T, d, q);
      r[0] = q[0] - meas[0]; r[1] = q[1] - meas[1]; r[2] = q[2] - meas[2];
      break;
    }
    case F_TERN: { /* previousPoint - H.inverse() * currentPoint */
      double Hi[12], l2H[3];
      oracle_pose_inverse(v[2], Hi);
      pose_transform_from(Hi, v[1], l2H);
      r[0] = v[0][0] - l2H[0]; r[1] = v[0][1] - l2H[1]; r[2] = v[0][2] - l2H[2];
      break;
    }
    case F_BTW: { /* Local(measured, a^-1 b) = Logmap(measured^-1 (a^-1 b)) */
      double ai[12], hx[12], zi[12], e[12];
      oracle_pose_inverse(v[0], ai);
      oracle_pose_compose(ai, v[1], hx);
      oracle_pose_inverse(meas, zi);
      oracle_pose_compose(zi, hx, e);
      oracle_pose_logmap(e, r);
      break;
    }
    case F_PRIOR: { /* -Local(x, prior) = -Logmap(x^-1 prior) */
      double xi[12], e[12], l[6];
      oracle_pose_inverse(v[0], xi);
      oracle_pose_compose(xi, meas, e);
      oracle_pose_logmap(e, l);
      for (int i = 0; i < 6; ++i) r[i] = -l[i];
      break;
    }
    case F_MP: { /* currentPoint - (currentPose * previousPose.inverse() * previousPoint) */
      double pi[12], c[12], q[3];
      oracle_pose_inverse(v[2], pi);
      oracle_pose_compose(v[3], pi, c);
      pose_transform_from(c, v[0], q);
      r[0] = v[1][0] - q[0]; r[1] = v[1][1] - q[1]; r[2] = v[1][2] - q[2];
      break;
    }
    case F_PS: {
      double i2[12], i1[12], a[12], b[12], ai[12], hx[12];
      oracle_pose_inverse(v[0], i2);
      oracle_pose_compose(v[1], i2, a);   /* k_2_H_k_1 = pose_k_1 * pose_k_2^-1 */
      oracle_pose_inverse(v[1], i1);
      oracle_pose_compose(v[2], i1, b);   /* k_1_H_k = pose_k * pose_k_1^-1 */
      oracle_pose_inverse(a, ai);
      oracle_pose_compose(ai, b, hx);     /* Between(a, b) */
      oracle_pose_logmap(hx, r);          /* Local(Identity, hx) */
      break;
    }
  }
}

/* gtsam::numericalDerivative11 (central, delta = 1e-5) of residual wrt
   slot s, written into columns [col0, col0+dim) of J (d x cols) */
static void numerical_slot(int type, const double* const* v, const double* meas,
                           int s, double* J, int cols, int col0) {
  const double delta = 1e-5;
  const int d = kDim[type];
  double hx[6], y1[6], y2[6];
  residual(type, v, meas, hx);
  const double* vv[4] = {v[0], v[1], v[2], v[3]};
  double pert[12];
  const double factor = 1.0 / (2.0 * delta);
  const int ds = slot_dim(type, s);
  for (int j = 0; j < ds; ++j) {
    double dx[6] = {0, 0, 0, 0, 0, 0};
    double dy1[6], dy2[6];
    for (int sgn = 0; sgn < 2; ++sgn) {
      dx[j] = sgn == 0 ? delta : -delta;
      if (ds == 6) {
        pose_retract(v[s], dx, pert);
      } else {
        pert[0] = v[s][0] + dx[0]; pert[1] = v[s][1] + dx[1]; pert[2] = v[s][2] + dx[2];
      }
      vv[s] = pert;
      residual(type, vv, meas, sgn == 0 ? y1 : y2);
      vv[s] = v[s];
    }
    for (int i = 0; i < d; ++i) { dy1[i] = y1[i] - hx[i]; dy2[i] = y2[i] - hx[i]; }
    for (int i = 0; i < d; ++i) J[i * cols + col0 + j] = (dy1[i] - dy2[i]) * factor;
  }
}

/* residual + Jacobians (unwhitened), J is d x cols row-major */
static void eval_factor(int type, const double* const* v, const double* meas,
                        double* r, double* J) {
  const int cols = oracle_factor_cols(type);
  switch (type) {
    case F_P2P: {
      /* Pose3::transformTo: Hself = [skew(q) | -I], Hpoint = R^T */
      residual(type, v, meas, r);
      const double* T = v[0];
      double d[3] = {v[1][0] - T[9], v[1][1] - T[10], v[1][2] - T[11]};
      double q[3];
      m3_tmv(T, d, q);
      const double wx = q[0], wy = q[1], wz = q[2];
      const double Hs[18] = {0.0, -wz, +wy, -1.0, 0.0, 0.0,
                             +wz, 0.0, -wx, 0.0, -1.0, 0.0,
                             -wy, +wx, 0.0, 0.0, 0.0, -1.0};
      for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 6; ++j) J[i * cols + j] = Hs[6 * i + j];
        for (int j = 0; j < 3; ++j) J[i * cols + 6 + j] = T[3 * j + i];
      }
      break;
    }
    case F_TERN: {
      /* LandmarkMotionTernaryFactor.cc:43-69 */
      residual(type, v, meas, r);
      double Hi[12], q[3];
      oracle_pose_inverse(v[2], Hi);
      pose_transform_from(Hi, v[1], q);
      memset(J, 0, 3 * cols * sizeof(double));
      for (int i = 0; i < 3; ++i) {
        J[i * cols + i] = 1.0;                                  /* J1 = I   */
        for (int j = 0; j < 3; ++j) J[i * cols + 3 + j] = -Hi[3 * i + j]; /* J2 */
        J[i * cols + 6 + 3 + i] = 1.0;                          /* J3 [.|I] */
      }
      J[0 * cols + 6 + 1] = q[2];  J[0 * cols + 6 + 2] = -q[1];
      J[1 * cols + 6 + 0] = -q[2]; J[1 * cols + 6 + 2] = q[0];
      J[2 * cols + 6 + 0] = q[1];  J[2 * cols + 6 + 1] = -q[0];
      break;
    }
    case F_BTW: {
      /* LieGroup::between: H1 = -hx^-1.AdjointMap(), H2 = I (the fast
         BetweenFactor Jacobians, GTSAM_SLOW_BUT_CORRECT_BETWEENFACTOR off) */
      residual(type, v, meas, r);
      double ai[12], hx[12], hxi[12], Ad[36];
      oracle_pose_inverse(v[0], ai);
      oracle_pose_compose(ai, v[1], hx);
      oracle_pose_inverse(hx, hxi);
      pose_adjoint(hxi, Ad);
      for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
          J[i * cols + j] = -Ad[6 * i + j];
          J[i * cols + 6 + j] = (i == j) ? 1.0 : 0.0;
        }
      break;
    }
    case F_PRIOR: {
      /* PriorFactor::evaluateError: H = I, r = -Local(x, prior) */
      residual(type, v, meas, r);
      for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) J[i * cols + j] = (i == j) ? 1.0 : 0.0;
      break;
    }
    case F_MP:
    case F_PS: {
      int col0 = 0;
      for (int s = 0; s < kNKeys[type]; ++s) {
        numerical_slot(type, v, meas, s, J, cols, col0);
        col0 += slot_dim(type, s);
      }
      residual(type, v, meas, r);
      break;
    }
  }
}

int oracle_eval_factor(int type, const double* vars, const double* meas,
                       double* r, double* J) {
  if (type < 0 || type >= F_NT) return -1;
  const double* v[4] = {NULL, NULL, NULL, NULL};
  int off = 0;
  for (int s = 0; s < kNKeys[type]; ++s) {
    v[s] = vars + off;
    off += slot_vsize(type, s);
  }
  eval_factor(type, v, meas, r, J);
  return 0;
}

/* ------------------------------------------------------------------ */
/* Problem                                                             */
/* ------------------------------------------------------------------ */
typedef struct {
  int type;
  int var[4];          /* variable indices */
  double meas[12];
  double inv_sigma[6];
  double huber_k;      /* <= 0: Gaussian */
} factor_t;

typedef struct { uint64_t key; int idx; } keyidx_t;

typedef struct {
  int npts;
  int* pts;            /* variable indices of points, local order */
  int nnb;             /* neighbouring poses (reduced order) */
  int* nb;             /* reduced pose indices, ascending */
  double* C;           /* (3n)^2 Cholesky factor (lower) */
  double* W;           /* 3n x 6m */
  double* Y;           /* 3n x 6m = C^-1 W */
  double* gp;          /* 3n */
  double* v;           /* C^-1 gp */
} comp_t;

struct oracle_problem {
  size_t nvars;
  uint64_t* keys;
  uint8_t* kind;
  size_t* voff;        /* offset in data */
  size_t ndata;
  double* data;
  keyidx_t* sorted;
  size_t nf;
  factor_t* f;
  size_t nft[F_NT];
  int dense;
  /* control (oracle_set_reverse_sums): the Schur solve accumulates the
     factors and eliminates the point components in reverse order, which
     changes only the rounding of the reduced system */
  int reverse_sums;
  /* control (oracle_set_solve_ld): every damped solve of the LM in x87
     extended precision (solve_schur_ld): the exact-step trajectory that
     the deep-convergence free runs are compared with */
  int solve_ld;
  char err[256];
  /* structure for the Schur solve */
  int* comp_of;        /* per variable: component id (points) or -1 */
  int* red_of;         /* per variable: reduced pose index or -1 */
  int npose;
  int* pose_var;       /* reduced index -> variable */
  int ncomp;
  comp_t* comps;
  int* nb_local;       /* scratch: reduced pose -> local index in current comp */
  size_t ndim_red;
  size_t* first;       /* skyline: first column per reduced row (dims) */
  size_t* rowoff;      /* skyline: offset of row i */
  double* sky;
  double* gc;
  /* linearisation */
  double* A;           /* per factor: d x cols */
  double* b;           /* per factor: d */
  size_t* foffA;
  size_t* foffb;
  /* LM state */
  dynohip_lm_params prm;
  double lambda;
  double error;
  int iterations;
  int inner;
  int converged;
  dynohip_trace_entry* trace;
  size_t ntrace, captrace;
  /* threaded solve (oracle_set_threads) */
  int nthreads;
  struct pool_t* pool;
  size_t* comp_f_start;   /* factors touching each component (CSR) */
  int* comp_f;
};

static void set_err(oracle_problem* p, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(p->err, sizeof(p->err), fmt, ap);
  va_end(ap);
}
const char* oracle_last_error(const oracle_problem* p) { return p ? p->err : "null"; }
void oracle_set_dense(oracle_problem* p, int dense) { p->dense = dense; }
void oracle_set_reverse_sums(oracle_problem* p, int reverse) { p->reverse_sums = reverse; }
void oracle_set_solve_ld(oracle_problem* p, int on) { p->solve_ld = on; }

static int cmp_keyidx(const void* a, const void* b) {
  const keyidx_t* x = (const keyidx_t*)a;
  const keyidx_t* y = (const keyidx_t*)b;
  return x->key < y->key ? -1 : (x->key > y->key ? 1 : 0);
}
static int find_var(const oracle_problem* p, uint64_t key) {
  size_t lo = 0, hi = p->nvars;
  while (lo < hi) {
    size_t mid = (lo + hi) / 2;
    if (p->sorted[mid].key < key) lo = mid + 1;
    else hi = mid;
  }
  if (lo < p->nvars && p->sorted[lo].key == key) return p->sorted[lo].idx;
  return -1;
}


/* frame-ordered pose key: (frame, chr, label) */
static void pose_order_key(uint64_t key, uint64_t* frame, unsigned* chr, unsigned* label) {
  const unsigned c = (unsigned)(key >> 56);
  const unsigned l = (unsigned)((key >> 48) & 0xff);
  *chr = c;
  if (c > 0 && l > 0) { *label = l; *frame = key & ((1ULL << 48) - 1); }
  else { *label = 0; *frame = key & ((1ULL << 56) - 1); }
}
typedef struct { uint64_t frame; unsigned chr, label; uint64_t key; int var; } posesort_t;
static int cmp_posesort(const void* a, const void* b) {
  const posesort_t* x = (const posesort_t*)a;
  const posesort_t* y = (const posesort_t*)b;
  if (x->frame != y->frame) return x->frame < y->frame ? -1 : 1;
  if (x->chr != y->chr) return x->chr < y->chr ? -1 : 1;
  if (x->label != y->label) return x->label < y->label ? -1 : 1;
  if (x->key != y->key) return x->key < y->key ? -1 : 1;
  return 0;
}

static int uf_find(int* par, int x) {
  while (par[x] != x) { par[x] = par[par[x]]; x = par[x]; }
  return x;
}
static int cmp_int(const void* a, const void* b) {
  int x = *(const int*)a, y = *(const int*)b;
  return x < y ? -1 : (x > y ? 1 : 0);
}

static int build_structure(oracle_problem* p) {
  const size_t nv = p->nvars;
  p->comp_of = (int*)malloc(nv * sizeof(int));
  p->red_of = (int*)malloc(nv * sizeof(int));
  /* poses: frame order */
  posesort_t* ps = (posesort_t*)malloc(nv * sizeof(posesort_t));
  int np = 0;
  for (size_t i = 0; i < nv; ++i) {
    p->red_of[i] = -1;
    if (p->kind[i] == DYNOHIP_POSE3) {
      pose_order_key(p->keys[i], &ps[np].frame, &ps[np].chr, &ps[np].label);
      ps[np].key = p->keys[i];
      ps[np].var = (int)i;
      ++np;
    }
  }
  qsort(ps, (size_t)np, sizeof(posesort_t), cmp_posesort);
  p->npose = np;
  p->pose_var = (int*)malloc((size_t)(np > 0 ? np : 1) * sizeof(int));
  for (int i = 0; i < np; ++i) { p->pose_var[i] = ps[i].var; p->red_of[ps[i].var] = i; }
  free(ps);
  p->nb_local = (int*)malloc((size_t)(np > 0 ? np : 1) * sizeof(int));
  for (int i = 0; i < np; ++i) p->nb_local[i] = -1;
  /* point components: union-find over factors with >= 2 points */
  int* par = (int*)malloc(nv * sizeof(int));
  for (size_t i = 0; i < nv; ++i) par[i] = (int)i;
  for (size_t f = 0; f < p->nf; ++f) {
    const factor_t* F = &p->f[f];
    int first = -1;
    for (int s = 0; s < kNKeys[F->type]; ++s) {
      if (kSlotKind[F->type][s] != 1) continue;
      if (first < 0) first = F->var[s];
      else {
        int a = uf_find(par, first), b = uf_find(par, F->var[s]);
        if (a != b) par[a] = b;
      }
    }
  }
  int* root_comp = (int*)malloc(nv * sizeof(int));
  for (size_t i = 0; i < nv; ++i) root_comp[i] = -1;
  int nc = 0;
  for (size_t i = 0; i < nv; ++i) {
    p->comp_of[i] = -1;
    if (p->kind[i] != DYNOHIP_POINT3) continue;
    int r = uf_find(par, (int)i);
    if (root_comp[r] < 0) root_comp[r] = nc++;
    p->comp_of[i] = root_comp[r];
  }
  p->ncomp = nc;
  p->comps = (comp_t*)calloc((size_t)(nc > 0 ? nc : 1), sizeof(comp_t));
  for (size_t i = 0; i < nv; ++i)
    if (p->comp_of[i] >= 0) p->comps[p->comp_of[i]].npts++;
  for (int c = 0; c < nc; ++c) {
    p->comps[c].pts = (int*)malloc((size_t)p->comps[c].npts * sizeof(int));
    p->comps[c].npts = 0;
  }
  for (size_t i = 0; i < nv; ++i)
    if (p->comp_of[i] >= 0) {
      comp_t* C = &p->comps[p->comp_of[i]];
      C->pts[C->npts++] = (int)i;
    }
  /* point local index within component */
  int* local = (int*)malloc(nv * sizeof(int));
  for (int c = 0; c < nc; ++c)
    for (int k = 0; k < p->comps[c].npts; ++k) local[p->comps[c].pts[k]] = k;
  /* neighbour poses of each component */
  int* cnt = (int*)calloc((size_t)(nc > 0 ? nc : 1), sizeof(int));
  for (size_t f = 0; f < p->nf; ++f) {
    const factor_t* F = &p->f[f];
    int comp = -1;
    for (int s = 0; s < kNKeys[F->type]; ++s)
      if (kSlotKind[F->type][s] == 1) comp = p->comp_of[F->var[s]];
    if (comp < 0) continue;
    for (int s = 0; s < kNKeys[F->type]; ++s)
      if (kSlotKind[F->type][s] == 0) cnt[comp]++;
  }
  for (int c = 0; c < nc; ++c) {
    p->comps[c].nb = (int*)malloc((size_t)(cnt[c] > 0 ? cnt[c] : 1) * sizeof(int));
    p->comps[c].nnb = 0;
  }
  for (size_t f = 0; f < p->nf; ++f) {
    const factor_t* F = &p->f[f];
    int comp = -1;
    for (int s = 0; s < kNKeys[F->type]; ++s)
      if (kSlotKind[F->type][s] == 1) comp = p->comp_of[F->var[s]];
    if (comp < 0) continue;
    for (int s = 0; s < kNKeys[F->type]; ++s)
      if (kSlotKind[F->type][s] == 0) {
        comp_t* C = &p->comps[comp];
        C->nb[C->nnb++] = p->red_of[F->var[s]];
      }
  }
  for (int c = 0; c < nc; ++c) {
    comp_t* C = &p->comps[c];
    qsort(C->nb, (size_t)C->nnb, sizeof(int), cmp_int);
    int u = 0;
    for (int k = 0; k < C->nnb; ++k)
      if (u == 0 || C->nb[u - 1] != C->nb[k]) C->nb[u++] = C->nb[k];
    C->nnb = u;
    const size_t n3 = 3 * (size_t)C->npts, m6 = 6 * (size_t)C->nnb;
    C->C = (double*)malloc(n3 * n3 * sizeof(double));
    C->W = (double*)malloc((n3 * m6 > 0 ? n3 * m6 : 1) * sizeof(double));
    C->Y = (double*)malloc((n3 * m6 > 0 ? n3 * m6 : 1) * sizeof(double));
    C->gp = (double*)malloc(n3 * sizeof(double));
    C->v = (double*)malloc(n3 * sizeof(double));
  }
  free(cnt);
  free(local);
  free(root_comp);
  free(par);
  /* skyline envelope over reduced pose dims */
  const size_t nd = 6 * (size_t)np;
  p->ndim_red = nd;
  int* firstpose = (int*)malloc((size_t)(np > 0 ? np : 1) * sizeof(int));
  for (int i = 0; i < np; ++i) firstpose[i] = i;
  for (size_t f = 0; f < p->nf; ++f) {
    const factor_t* F = &p->f[f];
    int mn = 1 << 30;
    for (int s = 0; s < kNKeys[F->type]; ++s)
      if (kSlotKind[F->type][s] == 0 && p->red_of[F->var[s]] < mn) mn = p->red_of[F->var[s]];
    for (int s = 0; s < kNKeys[F->type]; ++s)
      if (kSlotKind[F->type][s] == 0) {
        int r = p->red_of[F->var[s]];
        if (mn < firstpose[r]) firstpose[r] = mn;
      }
  }
  for (int c = 0; c < nc; ++c) {
    const comp_t* C = &p->comps[c];
    if (C->nnb == 0) continue;
    int mn = C->nb[0];
    for (int k = 0; k < C->nnb; ++k)
      if (mn < firstpose[C->nb[k]]) firstpose[C->nb[k]] = mn;
  }
  p->first = (size_t*)malloc((nd > 0 ? nd : 1) * sizeof(size_t));
  p->rowoff = (size_t*)malloc((nd + 1) * sizeof(size_t));
  size_t off = 0;
  for (int i = 0; i < np; ++i)
    for (int r = 0; r < 6; ++r) {
      size_t row = 6 * (size_t)i + r;
      p->first[row] = 6 * (size_t)firstpose[i];
      p->rowoff[row] = off;
      off += row - p->first[row] + 1;
    }
  p->rowoff[nd] = off;
  free(firstpose);
  p->sky = (double*)malloc((off > 0 ? off : 1) * sizeof(double));
  p->gc = (double*)malloc((nd > 0 ? nd : 1) * sizeof(double));
  return 0;
}

static int add_block(oracle_problem* p, int type, const dynohip_factor_block* blk) {
  if (blk->n == 0) return 0;
  if (!blk->keys || !blk->sigmas) { set_err(p, "factor type %d: null keys/sigmas", type); return DYNOHIP_EINVAL; }
  if (kMeasDim[type] > 0 && !blk->measured) { set_err(p, "factor type %d: null measured", type); return DYNOHIP_EINVAL; }
  for (size_t i = 0; i < blk->n; ++i) {
    factor_t* F = &p->f[p->nf];
    memset(F, 0, sizeof(*F));
    F->type = type;
    for (int s = 0; s < kNKeys[type]; ++s) {
      uint64_t key = blk->keys[i * kNKeys[type] + s];
      int v = find_var(p, key);
      if (v < 0) { set_err(p, "factor type %d #%zu: key %llu has no value", type, i, (unsigned long long)key); return DYNOHIP_EKEY; }
      int want = kSlotKind[type][s] == 0 ? DYNOHIP_POSE3 : DYNOHIP_POINT3;
      if (p->kind[v] != want) { set_err(p, "factor type %d #%zu: key %llu has wrong kind", type, i, (unsigned long long)key); return DYNOHIP_EINVAL; }
      F->var[s] = v;
    }
    for (int k = 0; k < kMeasDim[type]; ++k) F->meas[k] = blk->measured[i * kMeasDim[type] + k];
    for (int k = 0; k < kDim[type]; ++k) {
      double s = blk->sigmas[i * kDim[type] + k];
      if (!(s > 0.0) || !isfinite(s)) { set_err(p, "factor type %d #%zu: bad sigma", type, i); return DYNOHIP_EINVAL; }
      F->inv_sigma[k] = 1.0 / s;
    }
    F->huber_k = blk->huber_k ? blk->huber_k[i] : 0.0;
    p->nf++;
  }
  p->nft[type] += blk->n;
  return 0;
}

int oracle_create(const dynohip_graph_view* g, const uint64_t* keys,
                  const uint8_t* kind, const double* data, size_t n,
                  oracle_problem** out) {
  oracle_problem* p = (oracle_problem*)calloc(1, sizeof(oracle_problem));
  *out = p;
  if (!g || (!keys && n) || (!kind && n) || (!data && n)) { set_err(p, "null argument"); return DYNOHIP_EINVAL; }
  p->nvars = n;
  p->keys = (uint64_t*)malloc((n ? n : 1) * sizeof(uint64_t));
  p->kind = (uint8_t*)malloc((n ? n : 1));
  p->voff = (size_t*)malloc((n ? n : 1) * sizeof(size_t));
  p->sorted = (keyidx_t*)malloc((n ? n : 1) * sizeof(keyidx_t));
  size_t off = 0;
  for (size_t i = 0; i < n; ++i) {
    p->keys[i] = keys[i];
    p->kind[i] = kind[i];
    if (kind[i] > 1) { set_err(p, "bad kind"); return DYNOHIP_EINVAL; }
    p->voff[i] = off;
    off += kind[i] == DYNOHIP_POSE3 ? 12 : 3;
    p->sorted[i].key = keys[i];
    p->sorted[i].idx = (int)i;
  }
  p->ndata = off;
  p->data = (double*)malloc((off ? off : 1) * sizeof(double));
  memcpy(p->data, data, off * sizeof(double));
  qsort(p->sorted, n, sizeof(keyidx_t), cmp_keyidx);
  for (size_t i = 1; i < n; ++i)
    if (p->sorted[i].key == p->sorted[i - 1].key) { set_err(p, "duplicate key"); return DYNOHIP_EINVAL; }
  const dynohip_factor_block* blocks[F_NT] = {&g->pose_to_point, &g->landmark_motion_ternary, &g->between,
                                              &g->prior, &g->landmark_motion_pose, &g->landmark_pose_smoothing};
  size_t total = 0;
  for (int t = 0; t < F_NT; ++t) total += blocks[t]->n;
  p->f = (factor_t*)malloc((total ? total : 1) * sizeof(factor_t));
  for (int t = 0; t < F_NT; ++t) {
    int rc = add_block(p, t, blocks[t]);
    if (rc) return rc;
  }
  p->foffA = (size_t*)malloc((p->nf ? p->nf : 1) * sizeof(size_t));
  p->foffb = (size_t*)malloc((p->nf ? p->nf : 1) * sizeof(size_t));
  size_t oa = 0, ob = 0;
  for (size_t f = 0; f < p->nf; ++f) {
    p->foffA[f] = oa;
    p->foffb[f] = ob;
    oa += (size_t)kDim[p->f[f].type] * oracle_factor_cols(p->f[f].type);
    ob += (size_t)kDim[p->f[f].type];
  }
  p->A = (double*)malloc((oa ? oa : 1) * sizeof(double));
  p->b = (double*)malloc((ob ? ob : 1) * sizeof(double));
  build_structure(p);
  dynohip_lm_params d;
  memset(&d, 0, sizeof(d));
  d.lambda_initial = 1e-5; d.lambda_factor = 10.0; d.lambda_upper_bound = 1e5;
  d.lambda_lower_bound = 0.0; d.min_model_fidelity = 1e-3; d.relative_error_tol = 1e-5;
  d.absolute_error_tol = 1e-5; d.error_tol = 0.0; d.max_iterations = 100;
  d.use_fixed_lambda_factor = 1;
  oracle_lm_reset(p, &d);
  return 0;
}

void oracle_destroy(oracle_problem* p) {
  if (!p) return;
  free(p->keys); free(p->kind); free(p->voff); free(p->sorted); free(p->data);
  free(p->f); free(p->foffA); free(p->foffb); free(p->A); free(p->b);
  free(p->comp_of); free(p->red_of); free(p->pose_var); free(p->nb_local);
  for (int c = 0; c < p->ncomp; ++c) {
    free(p->comps[c].pts); free(p->comps[c].nb); free(p->comps[c].C);
    free(p->comps[c].W); free(p->comps[c].Y); free(p->comps[c].gp); free(p->comps[c].v);
  }
  free(p->comps); free(p->first); free(p->rowoff); free(p->sky); free(p->gc);
  free(p->trace);
  oracle_set_threads(p, 1);
  free(p->comp_f_start); free(p->comp_f);
  free(p);
}

/* ------------------------------------------------------------------ */
/* Error and linearisation                                             */
/* ------------------------------------------------------------------ */
static void factor_vars(const oracle_problem* p, const double* data, const factor_t* F, const double** v) {
  for (int s = 0; s < 4; ++s) v[s] = NULL;
  for (int s = 0; s < kNKeys[F->type]; ++s) v[s] = data + p->voff[F->var[s]];
}

/* NoiseModelFactor::error: loss(squaredMahalanobisDistance(r)) */
static double factor_error(const oracle_problem* p, const double* data, const factor_t* F) {
  const double* v[4];
  factor_vars(p, data, F, v);
  double r[6];
  residual(F->type, v, F->meas, r);
  double d2 = 0.0;
  for (int i = 0; i < kDim[F->type]; ++i) {
    const double w = r[i] * F->inv_sigma[i];
    d2 += w * w;
  }
  if (F->huber_k > 0.0) {
    const double e = sqrt(d2);
    const double k = F->huber_k;
    return e <= k ? e * e / 2 : k * (e - (k / 2));
  }
  return 0.5 * d2;
}

static double graph_error_mt(const oracle_problem* p, const double* data);
static double graph_error(const oracle_problem* p, const double* data) {
  if (p->nthreads > 1) return graph_error_mt(p, data);
  double s = 0.0;
  for (size_t f = 0; f < p->nf; ++f) s += factor_error(p, data, &p->f[f]);
  return s;
}
double oracle_error(oracle_problem* p) { return graph_error(p, p->data); }

/* NoiseModelFactor::linearize: b = -r, whiten, Huber block reweight */
static void linearize_one(oracle_problem* p, size_t f) {
  const factor_t* F = &p->f[f];
  const double* v[4];
  factor_vars(p, p->data, F, v);
  const int d = kDim[F->type], cols = oracle_factor_cols(F->type);
  double* A = p->A + p->foffA[f];
  double* b = p->b + p->foffb[f];
  double r[6];
  eval_factor(F->type, v, F->meas, r, A);
  double n2 = 0.0;
  for (int i = 0; i < d; ++i) {
    b[i] = -r[i] * F->inv_sigma[i];
    for (int j = 0; j < cols; ++j) A[i * cols + j] *= F->inv_sigma[i];
    n2 += b[i] * b[i];
  }
  if (F->huber_k > 0.0) {
    const double e = sqrt(n2);
    const double w = e <= F->huber_k ? 1.0 : F->huber_k / e;
    const double sw = sqrt(w);
    for (int i = 0; i < d; ++i) {
      b[i] *= sw;
      for (int j = 0; j < cols; ++j) A[i * cols + j] *= sw;
    }
  }
}

static void linearize_all_mt(oracle_problem* p);
static void linearize_all(oracle_problem* p) {
  if (p->nthreads > 1) { linearize_all_mt(p); return; }
  for (size_t f = 0; f < p->nf; ++f) linearize_one(p, f);
}

size_t oracle_linearize_size(const oracle_problem* p) {
  size_t n = 0;
  for (size_t f = 0; f < p->nf; ++f)
    n += (size_t)kDim[p->f[f].type] * (oracle_factor_cols(p->f[f].type) + 1);
  return n;
}
int oracle_linearize(oracle_problem* p, double* out, size_t n_doubles) {
  if (n_doubles < oracle_linearize_size(p)) return DYNOHIP_EINVAL;
  linearize_all(p);
  size_t o = 0;
  for (size_t f = 0; f < p->nf; ++f) {
    const int d = kDim[p->f[f].type], cols = oracle_factor_cols(p->f[f].type);
    for (int i = 0; i < d; ++i) {
      for (int j = 0; j < cols; ++j) out[o++] = p->A[p->foffA[f] + (size_t)i * cols + j];
      out[o++] = p->b[p->foffb[f] + i];
    }
  }
  return 0;
}

/* JacobianFactor::error summed: 0.5 * || A delta - b ||^2 ; delta per
   variable in value-data layout (6 per pose, 3 per point) via doff */
/* the squared residual rows e_i^2 of factor f (at rows[foffb[f]..]) */
static void linear_error_rows(const oracle_problem* p, size_t f, const double* delta, const size_t* doff,
                              double* rows) {
  const factor_t* F = &p->f[f];
  const int d = kDim[F->type], cols = oracle_factor_cols(F->type);
  const double* A = p->A + p->foffA[f];
  const double* b = p->b + p->foffb[f];
  for (int i = 0; i < d; ++i) {
    double acc = 0.0;
    if (delta) {
      int c = 0;
      for (int sl = 0; sl < kNKeys[F->type]; ++sl) {
        const double* dv = delta + doff[F->var[sl]];
        for (int j = 0; j < slot_dim(F->type, sl); ++j, ++c) acc += A[i * cols + c] * dv[j];
      }
    }
    const double e = acc - b[i];
    rows[p->foffb[f] + i] = e * e;
  }
}
static double linear_error_mt(const oracle_problem* p, const double* delta, const size_t* doff);
static double linear_error(const oracle_problem* p, const double* delta, const size_t* doff) {
  if (p->nthreads > 1) return linear_error_mt(p, delta, doff);
  double s = 0.0;
  for (size_t f = 0; f < p->nf; ++f) {
    const factor_t* F = &p->f[f];
    const int d = kDim[F->type], cols = oracle_factor_cols(F->type);
    const double* A = p->A + p->foffA[f];
    const double* b = p->b + p->foffb[f];
    for (int i = 0; i < d; ++i) {
      double acc = 0.0;
      if (delta) {
        int c = 0;
        for (int sl = 0; sl < kNKeys[F->type]; ++sl) {
          const double* dv = delta + doff[F->var[sl]];
          for (int j = 0; j < slot_dim(F->type, sl); ++j, ++c) acc += A[i * cols + c] * dv[j];
        }
      }
      const double e = acc - b[i];
      s += e * e;
    }
  }
  return 0.5 * s;
}

/* ------------------------------------------------------------------ */
/* Linear algebra                                                      */
/* ------------------------------------------------------------------ */
/* in-place lower Cholesky of an n x n row-major matrix; 0 if not PD */
static int chol_dense(double* A, size_t n) {
  for (size_t j = 0; j < n; ++j) {
    double d = A[j * n + j];
    for (size_t k = 0; k < j; ++k) d -= A[j * n + k] * A[j * n + k];
    if (!(d > 0.0) || !isfinite(d)) return 0;
    const double ljj = sqrt(d);
    A[j * n + j] = ljj;
    for (size_t i = j + 1; i < n; ++i) {
      double s = A[i * n + j];
      for (size_t k = 0; k < j; ++k) s -= A[i * n + k] * A[j * n + k];
      A[i * n + j] = s / ljj;
    }
  }
  return 1;
}
/* solve L L^T x = b in place (b: n x nrhs, row-major, column stride nrhs) */
static void chol_solve(const double* L, size_t n, double* B, size_t nrhs) {
  for (size_t c = 0; c < nrhs; ++c) {
    for (size_t i = 0; i < n; ++i) {
      double s = B[i * nrhs + c];
      for (size_t k = 0; k < i; ++k) s -= L[i * n + k] * B[k * nrhs + c];
      B[i * nrhs + c] = s / L[i * n + i];
    }
    for (size_t ii = n; ii-- > 0;) {
      double s = B[ii * nrhs + c];
      for (size_t k = ii + 1; k < n; ++k) s -= L[k * n + ii] * B[k * nrhs + c];
      B[ii * nrhs + c] = s / L[ii * n + ii];
    }
  }
}

/* global variable ordering for dense / delta layout */
static size_t var_dim(const oracle_problem* p, int v) { return p->kind[v] == DYNOHIP_POSE3 ? 6 : 3; }

/* Solve (A^T A + lambda I) delta = A^T b. delta laid out with doff.
   returns 1 solved, 0 indefinite */
static int solve_dense(oracle_problem* p, double lambda, double* delta, const size_t* doff, size_t N) {
  double* H = (double*)calloc(N * N, sizeof(double));
  double* g = (double*)calloc(N, sizeof(double));
  for (size_t f = 0; f < p->nf; ++f) {
    const factor_t* F = &p->f[f];
    const int d = kDim[F->type], cols = oracle_factor_cols(F->type);
    const double* A = p->A + p->foffA[f];
    const double* b = p->b + p->foffb[f];
    int c0 = 0;
    for (int sa = 0; sa < kNKeys[F->type]; ++sa) {
      const int da = slot_dim(F->type, sa);
      const size_t oa = doff[F->var[sa]];
      for (int ia = 0; ia < da; ++ia)
        for (int r = 0; r < d; ++r) g[oa + ia] += A[r * cols + c0 + ia] * b[r];
      int c1 = 0;
      for (int sb = 0; sb < kNKeys[F->type]; ++sb) {
        const int db = slot_dim(F->type, sb);
        const size_t ob = doff[F->var[sb]];
        for (int ia = 0; ia < da; ++ia)
          for (int ib = 0; ib < db; ++ib) {
            double s = 0.0;
            for (int r = 0; r < d; ++r) s += A[r * cols + c0 + ia] * A[r * cols + c1 + ib];
            H[(oa + ia) * N + ob + ib] += s;
          }
        c1 += db;
      }
      c0 += da;
    }
  }
  for (size_t i = 0; i < N; ++i) H[i * N + i] += lambda;
  int ok = chol_dense(H, N);
  if (ok) {
    chol_solve(H, N, g, 1);
    memcpy(delta, g, N * sizeof(double));
  }
  free(H);
  free(g);
  return ok;
}

static double* sky_at(oracle_problem* p, size_t i, size_t j) { /* i >= j */
  return &p->sky[p->rowoff[i] + (j - p->first[i])];
}

static int solve_schur(oracle_problem* p, double lambda, double* delta, const size_t* doff) {
  const size_t nd = p->ndim_red;
  memset(p->sky, 0, p->rowoff[nd] * sizeof(double));
  memset(p->gc, 0, nd * sizeof(double));
  int* local = (int*)malloc(p->nvars * sizeof(int));
  for (int c = 0; c < p->ncomp; ++c) {
    comp_t* C = &p->comps[c];
    const size_t n3 = 3 * (size_t)C->npts, m6 = 6 * (size_t)C->nnb;
    memset(C->C, 0, n3 * n3 * sizeof(double));
    memset(C->W, 0, n3 * m6 * sizeof(double));
    memset(C->gp, 0, n3 * sizeof(double));
    for (int k = 0; k < C->npts; ++k) local[C->pts[k]] = k;
  }
  /* accumulate normal-equation blocks */
  for (size_t f0 = 0; f0 < p->nf; ++f0) {
    const size_t f = p->reverse_sums ? p->nf - 1 - f0 : f0;
    const factor_t* F = &p->f[f];
    const int d = kDim[F->type], cols = oracle_factor_cols(F->type), nk = kNKeys[F->type];
    const double* A = p->A + p->foffA[f];
    const double* b = p->b + p->foffb[f];
    int comp = -1;
    for (int s = 0; s < nk; ++s)
      if (kSlotKind[F->type][s] == 1) comp = p->comp_of[F->var[s]];
    comp_t* C = comp >= 0 ? &p->comps[comp] : NULL;
    if (C)
      for (int k = 0; k < C->nnb; ++k) p->nb_local[C->nb[k]] = k;
    int c0 = 0;
    for (int sa = 0; sa < nk; ++sa) {
      const int da = slot_dim(F->type, sa);
      const int va = F->var[sa];
      const int pa = kSlotKind[F->type][sa] == 1;
      /* gradient */
      for (int ia = 0; ia < da; ++ia) {
        double s = 0.0;
        for (int r = 0; r < d; ++r) s += A[r * cols + c0 + ia] * b[r];
        if (pa) C->gp[3 * local[va] + ia] += s;
        else p->gc[6 * (size_t)p->red_of[va] + ia] += s;
      }
      int c1 = 0;
      for (int sb = 0; sb < nk; ++sb) {
        const int db = slot_dim(F->type, sb);
        const int vb = F->var[sb];
        const int pb = kSlotKind[F->type][sb] == 1;
        for (int ia = 0; ia < da; ++ia)
          for (int ib = 0; ib < db; ++ib) {
            double s = 0.0;
            for (int r = 0; r < d; ++r) s += A[r * cols + c0 + ia] * A[r * cols + c1 + ib];
            if (pa && pb) {
              C->C[(3 * (size_t)local[va] + ia) * (3 * (size_t)C->npts) + 3 * (size_t)local[vb] + ib] += s;
            } else if (pa && !pb) {
              C->W[(3 * (size_t)local[va] + ia) * (6 * (size_t)C->nnb) + 6 * (size_t)p->nb_local[p->red_of[vb]] + ib] += s;
            } else if (!pa && !pb) {
              size_t gi = 6 * (size_t)p->red_of[va] + ia, gj = 6 * (size_t)p->red_of[vb] + ib;
              if (gi >= gj) *sky_at(p, gi, gj) += s;
            }
          }
        c1 += db;
      }
      c0 += da;
    }
  }
  free(local);
  for (size_t i = 0; i < nd; ++i) *sky_at(p, i, i) += lambda;
  /* eliminate point components */
  for (int c0 = 0; c0 < p->ncomp; ++c0) {
    const int c = p->reverse_sums ? p->ncomp - 1 - c0 : c0;
    comp_t* C = &p->comps[c];
    const size_t n3 = 3 * (size_t)C->npts, m6 = 6 * (size_t)C->nnb;
    for (size_t i = 0; i < n3; ++i) C->C[i * n3 + i] += lambda;
    /* C was accumulated fully (both triangles); chol uses the lower part */
    if (!chol_dense(C->C, n3)) return 0;
    memcpy(C->Y, C->W, n3 * m6 * sizeof(double));
    chol_solve(C->C, n3, C->Y, m6);
    memcpy(C->v, C->gp, n3 * sizeof(double));
    chol_solve(C->C, n3, C->v, 1);
    for (int a = 0; a < C->nnb; ++a)
      for (int ia = 0; ia < 6; ++ia) {
        const size_t gi = 6 * (size_t)C->nb[a] + ia;
        double s = 0.0;
        for (size_t k = 0; k < n3; ++k) s += C->W[k * m6 + 6 * a + ia] * C->v[k];
        p->gc[gi] -= s;
        for (int bb = 0; bb <= a; ++bb)
          for (int ib = 0; ib < 6; ++ib) {
            const size_t gj = 6 * (size_t)C->nb[bb] + ib;
            if (gj > gi) continue;
            double t = 0.0;
            for (size_t k = 0; k < n3; ++k) t += C->W[k * m6 + 6 * a + ia] * C->Y[k * m6 + 6 * bb + ib];
            *sky_at(p, gi, gj) -= t;
          }
      }
  }
  /* envelope Cholesky of the reduced system (row-oriented) */
  for (size_t i = 0; i < nd; ++i) {
    const size_t fi = p->first[i];
    for (size_t j = fi; j <= i; ++j) {
      const size_t fj = p->first[j];
      const size_t k0 = fi > fj ? fi : fj;
      double s = *sky_at(p, i, j);
      for (size_t k = k0; k < j; ++k) s -= *sky_at(p, i, k) * *sky_at(p, j, k);
      if (j == i) {
        if (!(s > 0.0) || !isfinite(s)) return 0;
        *sky_at(p, i, i) = sqrt(s);
      } else {
        *sky_at(p, i, j) = s / *sky_at(p, j, j);
      }
    }
  }
  /* forward / backward substitution */
  double* x = (double*)malloc((nd ? nd : 1) * sizeof(double));
  for (size_t i = 0; i < nd; ++i) {
    double s = p->gc[i];
    for (size_t k = p->first[i]; k < i; ++k) s -= *sky_at(p, i, k) * x[k];
    x[i] = s / *sky_at(p, i, i);
  }
  for (size_t ii = nd; ii-- > 0;) {
    x[ii] /= *sky_at(p, ii, ii);
    const double xi = x[ii];
    for (size_t k = p->first[ii]; k < ii; ++k) x[k] -= *sky_at(p, ii, k) * xi;
  }
  for (int r = 0; r < p->npose; ++r)
    for (int k = 0; k < 6; ++k) delta[doff[p->pose_var[r]] + k] = x[6 * (size_t)r + k];
  free(x);
  /* back-substitute points: dp = C^-1 (gp - W dc) */
  for (int c = 0; c < p->ncomp; ++c) {
    comp_t* C = &p->comps[c];
    const size_t n3 = 3 * (size_t)C->npts, m6 = 6 * (size_t)C->nnb;
    double* rhs = (double*)malloc(n3 * sizeof(double));
    for (size_t k = 0; k < n3; ++k) {
      double s = C->gp[k];
      for (int a = 0; a < C->nnb; ++a)
        for (int ia = 0; ia < 6; ++ia)
          s -= C->W[k * m6 + 6 * a + ia] * delta[doff[p->pose_var[C->nb[a]]] + ia];
      rhs[k] = s;
    }
    chol_solve(C->C, n3, rhs, 1);
    for (int k = 0; k < C->npts; ++k)
      for (int j = 0; j < 3; ++j) delta[doff[C->pts[k]] + j] = rhs[3 * k + j];
    free(rhs);
  }
  return 1;
}

static size_t make_doff(const oracle_problem* p, size_t* doff) {
  size_t o = 0;
  for (size_t i = 0; i < p->nvars; ++i) { doff[i] = o; o += var_dim(p, (int)i); }
  return o;
}

static int solve_schur_mt(oracle_problem* p, double lambda, double* delta, const size_t* doff);
static int solve_schur_ld(oracle_problem* p, double lambda, double* delta, const size_t* doff);
static int solve_system(oracle_problem* p, double lambda, double* delta, const size_t* doff, size_t N) {
  if (p->solve_ld) return solve_schur_ld(p, lambda, delta, doff);
  if (p->dense) return solve_dense(p, lambda, delta, doff, N);
  if (p->nthreads > 1 && !p->reverse_sums) return solve_schur_mt(p, lambda, delta, doff);
  return solve_schur(p, lambda, delta, doff);
}

/* The same Schur solve with every sum, product and factorisation of the
   solve in x87 extended precision (64-bit significand, eps 5.4e-20): a
   reference for the deep-convergence steps, whose reduced systems are
   conditioned beyond 1/eps of double. The linearisation is
   the double one (the records), only the solve is extended. Serial. */
typedef long double ldbl;
static int chol_dense_ld(ldbl* A, size_t n) {
  for (size_t j = 0; j < n; ++j) {
    ldbl d = A[j * n + j];
    for (size_t k = 0; k < j; ++k) d -= A[j * n + k] * A[j * n + k];
    if (!(d > 0.0L)) return 0;
    const ldbl ljj = sqrtl(d);
    A[j * n + j] = ljj;
    for (size_t i = j + 1; i < n; ++i) {
      ldbl s = A[i * n + j];
      for (size_t k = 0; k < j; ++k) s -= A[i * n + k] * A[j * n + k];
      A[i * n + j] = s / ljj;
    }
  }
  return 1;
}
static void chol_solve_ld(const ldbl* L, size_t n, ldbl* B, size_t nrhs) {
  for (size_t c = 0; c < nrhs; ++c) {
    for (size_t i = 0; i < n; ++i) {
      ldbl s = B[i * nrhs + c];
      for (size_t k = 0; k < i; ++k) s -= L[i * n + k] * B[k * nrhs + c];
      B[i * nrhs + c] = s / L[i * n + i];
    }
    for (size_t ii = n; ii-- > 0;) {
      ldbl s = B[ii * nrhs + c];
      for (size_t k = ii + 1; k < n; ++k) s -= L[k * n + ii] * B[k * nrhs + c];
      B[ii * nrhs + c] = s / L[ii * n + ii];
    }
  }
}
static int solve_schur_ld(oracle_problem* p, double lambda, double* delta, const size_t* doff) {
  const size_t nd = p->ndim_red, nsky = p->rowoff[nd];
  ldbl* sky = (ldbl*)calloc(nsky ? nsky : 1, sizeof(ldbl));
  ldbl* gc = (ldbl*)calloc(nd ? nd : 1, sizeof(ldbl));
  ldbl** cC = (ldbl**)calloc((size_t)p->ncomp + 1, sizeof(ldbl*));
  ldbl** cW = (ldbl**)calloc((size_t)p->ncomp + 1, sizeof(ldbl*));
  ldbl** cg = (ldbl**)calloc((size_t)p->ncomp + 1, sizeof(ldbl*));
  int* local = (int*)malloc((p->nvars ? p->nvars : 1) * sizeof(int));
  int ok = 1;
#define SKY(i, j) sky[p->rowoff[i] + ((j) - p->first[i])]
  for (int c = 0; c < p->ncomp; ++c) {
    comp_t* C = &p->comps[c];
    const size_t n3 = 3 * (size_t)C->npts, m6 = 6 * (size_t)C->nnb;
    cC[c] = (ldbl*)calloc(n3 * n3 + 1, sizeof(ldbl));
    cW[c] = (ldbl*)calloc(n3 * m6 + 1, sizeof(ldbl));
    cg[c] = (ldbl*)calloc(n3 + 1, sizeof(ldbl));
    for (int k = 0; k < C->npts; ++k) local[C->pts[k]] = k;
  }
  for (size_t f = 0; f < p->nf; ++f) {
    const factor_t* F = &p->f[f];
    const int d = kDim[F->type], cols = oracle_factor_cols(F->type), nk = kNKeys[F->type];
    const double* A = p->A + p->foffA[f];
    const double* b = p->b + p->foffb[f];
    int comp = -1;
    for (int sl = 0; sl < nk; ++sl)
      if (kSlotKind[F->type][sl] == 1) comp = p->comp_of[F->var[sl]];
    comp_t* C = comp >= 0 ? &p->comps[comp] : NULL;
    if (C)
      for (int k = 0; k < C->nnb; ++k) p->nb_local[C->nb[k]] = k;
    int c0 = 0;
    for (int sa = 0; sa < nk; ++sa) {
      const int da = slot_dim(F->type, sa), va = F->var[sa], pa = kSlotKind[F->type][sa] == 1;
      for (int ia = 0; ia < da; ++ia) {
        ldbl sg = 0.0L;
        for (int r = 0; r < d; ++r) sg += (ldbl)A[r * cols + c0 + ia] * (ldbl)b[r];
        if (pa) cg[comp][3 * local[va] + ia] += sg;
        else gc[6 * (size_t)p->red_of[va] + ia] += sg;
      }
      int c1 = 0;
      for (int sb = 0; sb < nk; ++sb) {
        const int db = slot_dim(F->type, sb), vb = F->var[sb], pb = kSlotKind[F->type][sb] == 1;
        for (int ia = 0; ia < da; ++ia)
          for (int ib = 0; ib < db; ++ib) {
            ldbl t = 0.0L;
            for (int r = 0; r < d; ++r) t += (ldbl)A[r * cols + c0 + ia] * (ldbl)A[r * cols + c1 + ib];
            if (pa && pb) {
              cC[comp][(3 * (size_t)local[va] + ia) * (3 * (size_t)C->npts) + 3 * (size_t)local[vb] + ib] += t;
            } else if (pa && !pb) {
              cW[comp][(3 * (size_t)local[va] + ia) * (6 * (size_t)C->nnb) + 6 * (size_t)p->nb_local[p->red_of[vb]] + ib] += t;
            } else if (!pa && !pb) {
              const size_t gi = 6 * (size_t)p->red_of[va] + ia, gj = 6 * (size_t)p->red_of[vb] + ib;
              if (gi >= gj) SKY(gi, gj) += t;
            }
          }
        c1 += db;
      }
      c0 += da;
    }
  }
  for (size_t i = 0; i < nd; ++i) SKY(i, i) += (ldbl)lambda;
  ldbl** cY = (ldbl**)calloc((size_t)p->ncomp + 1, sizeof(ldbl*));
  for (int c = 0; c < p->ncomp && ok; ++c) {
    comp_t* C = &p->comps[c];
    const size_t n3 = 3 * (size_t)C->npts, m6 = 6 * (size_t)C->nnb;
    for (size_t i = 0; i < n3; ++i) cC[c][i * n3 + i] += (ldbl)lambda;
    if (!chol_dense_ld(cC[c], n3)) { ok = 0; break; }
    cY[c] = (ldbl*)malloc((n3 * m6 + 1) * sizeof(ldbl));
    memcpy(cY[c], cW[c], n3 * m6 * sizeof(ldbl));
    chol_solve_ld(cC[c], n3, cY[c], m6);
    ldbl* v = (ldbl*)malloc((n3 + 1) * sizeof(ldbl));
    memcpy(v, cg[c], n3 * sizeof(ldbl));
    chol_solve_ld(cC[c], n3, v, 1);
    for (int a = 0; a < C->nnb; ++a)
      for (int ia = 0; ia < 6; ++ia) {
        const size_t gi = 6 * (size_t)C->nb[a] + ia;
        ldbl sv = 0.0L;
        for (size_t k = 0; k < n3; ++k) sv += cW[c][k * m6 + 6 * a + ia] * v[k];
        gc[gi] -= sv;
        for (int bb = 0; bb <= a; ++bb)
          for (int ib = 0; ib < 6; ++ib) {
            const size_t gj = 6 * (size_t)C->nb[bb] + ib;
            if (gj > gi) continue;
            ldbl t = 0.0L;
            for (size_t k = 0; k < n3; ++k) t += cW[c][k * m6 + 6 * a + ia] * cY[c][k * m6 + 6 * bb + ib];
            SKY(gi, gj) -= t;
          }
      }
    free(v);
  }
  for (size_t i = 0; i < nd && ok; ++i) {
    const size_t fi = p->first[i];
    for (size_t j = fi; j <= i; ++j) {
      const size_t fj = p->first[j], k0 = fi > fj ? fi : fj;
      ldbl t = SKY(i, j);
      for (size_t k = k0; k < j; ++k) t -= SKY(i, k) * SKY(j, k);
      if (j == i) {
        if (!(t > 0.0L)) { ok = 0; break; }
        SKY(i, i) = sqrtl(t);
      } else {
        SKY(i, j) = t / SKY(j, j);
      }
    }
  }
  if (ok) {
    ldbl* x = (ldbl*)malloc((nd ? nd : 1) * sizeof(ldbl));
    for (size_t i = 0; i < nd; ++i) {
      ldbl t = gc[i];
      for (size_t k = p->first[i]; k < i; ++k) t -= SKY(i, k) * x[k];
      x[i] = t / SKY(i, i);
    }
    for (size_t ii = nd; ii-- > 0;) {
      x[ii] /= SKY(ii, ii);
      const ldbl xi = x[ii];
      for (size_t k = p->first[ii]; k < ii; ++k) x[k] -= SKY(ii, k) * xi;
    }
    for (int r = 0; r < p->npose; ++r)
      for (int k = 0; k < 6; ++k) delta[doff[p->pose_var[r]] + k] = (double)x[6 * (size_t)r + k];
    for (int c = 0; c < p->ncomp; ++c) {
      comp_t* C = &p->comps[c];
      const size_t n3 = 3 * (size_t)C->npts, m6 = 6 * (size_t)C->nnb;
      ldbl* rhs = (ldbl*)malloc((n3 + 1) * sizeof(ldbl));
      for (size_t k = 0; k < n3; ++k) {
        ldbl t = cg[c][k];
        for (int a = 0; a < C->nnb; ++a)
          for (int ia = 0; ia < 6; ++ia) t -= cW[c][k * m6 + 6 * a + ia] * x[6 * (size_t)C->nb[a] + ia];
        rhs[k] = t;
      }
      chol_solve_ld(cC[c], n3, rhs, 1);
      for (int k = 0; k < C->npts; ++k)
        for (int j = 0; j < 3; ++j) delta[doff[C->pts[k]] + j] = (double)rhs[3 * k + j];
      free(rhs);
    }
    free(x);
  }
#undef SKY
  for (int c = 0; c < p->ncomp; ++c) { free(cC[c]); free(cW[c]); free(cg[c]); free(cY[c]); }
  free(cC); free(cW); free(cg); free(cY); free(local); free(sky); free(gc);
  return ok;
}

int oracle_solve_damped_ld(oracle_problem* p, double lambda, double* delta_out, size_t n_doubles) {
  size_t* doff = (size_t*)malloc((p->nvars ? p->nvars : 1) * sizeof(size_t));
  size_t N = make_doff(p, doff);
  if (n_doubles < N) { free(doff); return DYNOHIP_EINVAL; }
  linearize_all(p);
  int ok = solve_schur_ld(p, lambda, delta_out, doff);
  free(doff);
  return ok;
}

int oracle_solve_damped(oracle_problem* p, double lambda, double* delta_out, size_t n_doubles) {
  size_t* doff = (size_t*)malloc((p->nvars ? p->nvars : 1) * sizeof(size_t));
  size_t N = make_doff(p, doff);
  if (n_doubles < N) { free(doff); return DYNOHIP_EINVAL; }
  linearize_all(p);
  int ok = solve_system(p, lambda, delta_out, doff, N);
  free(doff);
  return ok;
}

/* ------------------------------------------------------------------ */
/* Levenberg–Marquardt (GTSAM 4.2.0 LevenbergMarquardtOptimizer)       */
/* ------------------------------------------------------------------ */
int oracle_lm_reset(oracle_problem* p, const dynohip_lm_params* prm) {
  if (prm->diagonal_damping || !prm->use_fixed_lambda_factor) {
    set_err(p, "only diagonalDamping=false, useFixedLambdaFactor=true supported");
    return DYNOHIP_EINVAL;
  }
  p->prm = *prm;
  p->lambda = prm->lambda_initial;
  p->error = graph_error(p, p->data);
  p->iterations = 0;
  p->inner = 0;
  p->converged = 0;
  p->ntrace = 0;
  return 0;
}

static void push_trace(oracle_problem* p, const dynohip_trace_entry* e) {
  if (p->ntrace == p->captrace) {
    p->captrace = p->captrace ? 2 * p->captrace : 64;
    p->trace = (dynohip_trace_entry*)realloc(p->trace, p->captrace * sizeof(dynohip_trace_entry));
  }
  p->trace[p->ntrace++] = *e;
}

static void retract_all(const oracle_problem* p, const double* delta, const size_t* doff, double* out) {
  for (size_t i = 0; i < p->nvars; ++i) {
    const double* x = p->data + p->voff[i];
    const double* d = delta + doff[i];
    double* o = out + p->voff[i];
    if (p->kind[i] == DYNOHIP_POSE3) pose_retract(x, d, o);
    else { o[0] = x[0] + d[0]; o[1] = x[1] + d[1]; o[2] = x[2] + d[2]; }
  }
}

/* one outer iteration: LevenbergMarquardtOptimizer::iterate() */
static int lm_iterate(oracle_problem* p) {
  size_t* doff = (size_t*)malloc((p->nvars ? p->nvars : 1) * sizeof(size_t));
  const size_t N = make_doff(p, doff);
  double* delta = (double*)calloc(N ? N : 1, sizeof(double));
  double* newdata = (double*)malloc((p->ndata ? p->ndata : 1) * sizeof(double));
  linearize_all(p);
  const double oldLin = linear_error(p, NULL, doff);
  for (;;) {
    /* tryLambda */
    dynohip_trace_entry te;
    memset(&te, 0, sizeof(te));
    te.outer_iteration = p->iterations;
    te.lambda = p->lambda;
    te.current_error = p->error;
    te.new_error = INFINITY;
    te.old_linear_error = oldLin;
    int step_ok = 0, stop = 0;
    double modelFidelity = 0.0, newError = INFINITY;
    const int solved = solve_system(p, p->lambda, delta, doff, N);
    te.solved = solved;
    if (solved) {
      const double newLin = linear_error(p, delta, doff);
      te.new_linear_error = newLin;
      const double linChange = oldLin - newLin;
      if (linChange >= 0) {
        retract_all(p, delta, doff, newdata);
        newError = graph_error(p, newdata);
        te.new_error = newError;
        const double costChange = p->error - newError;
        if (linChange > DBL_EPSILON * oldLin) {
          modelFidelity = costChange / linChange;
          step_ok = modelFidelity > p->prm.min_model_fidelity;
        }
        const double minAbs = p->prm.relative_error_tol * p->error;
        if (fabs(costChange) < minAbs) stop = 1;
      }
    }
    te.model_fidelity = modelFidelity;
    te.accepted = step_ok;
    te.stop = stop;
    push_trace(p, &te);
    if (step_ok) {
      memcpy(p->data, newdata, p->ndata * sizeof(double));
      p->error = newError;
      p->lambda /= p->prm.lambda_factor;
      if (p->lambda < p->prm.lambda_lower_bound) p->lambda = p->prm.lambda_lower_bound;
      p->iterations++;
      p->inner++;
      break;
    } else if (!stop) {
      p->lambda *= p->prm.lambda_factor;
      p->inner++;
      if (p->lambda >= p->prm.lambda_upper_bound) break;
    } else {
      break;
    }
  }
  free(doff);
  free(delta);
  free(newdata);
  return 0;
}

static void fill_summary(const oracle_problem* p, double initial, dynohip_lm_summary* s) {
  if (!s) return;
  s->iterations = p->iterations;
  s->inner_iterations = p->inner;
  s->initial_error = initial;
  s->final_error = p->error;
  s->final_lambda = p->lambda;
  s->converged = p->converged;
}

int oracle_iterate(oracle_problem* p, dynohip_lm_summary* s) {
  const double e0 = p->error;
  lm_iterate(p);
  fill_summary(p, e0, s);
  return 0;
}

/* NonlinearOptimizer::defaultOptimize + checkConvergence */
static int check_convergence(const dynohip_lm_params* prm, double cur, double nw) {
  if (nw <= prm->error_tol) return 1;
  const double absd = cur - nw;
  const double reld = absd / cur;
  return (reld <= prm->relative_error_tol) || (absd <= prm->absolute_error_tol);
}

int oracle_optimize(oracle_problem* p, const dynohip_lm_params* prm, dynohip_lm_summary* s) {
  int rc = oracle_lm_reset(p, prm);
  if (rc) return rc;
  const double initial = p->error;
  double currentError = p->error;
  if (currentError <= prm->error_tol || p->iterations >= prm->max_iterations) {
    p->converged = currentError <= prm->error_tol;
    fill_summary(p, initial, s);
    return 0;
  }
  double newError = currentError;
  do {
    currentError = newError;
    lm_iterate(p);
    newError = p->error;
    p->converged = check_convergence(prm, currentError, newError);
  } while (p->iterations < prm->max_iterations && !p->converged && isfinite(currentError));
  fill_summary(p, initial, s);
  return 0;
}

int oracle_get_values(const oracle_problem* p, double* out, size_t n_doubles) {
  if (n_doubles < p->ndata) return DYNOHIP_EINVAL;
  memcpy(out, p->data, p->ndata * sizeof(double));
  return 0;
}
int oracle_set_values_data(oracle_problem* p, const double* data, size_t n_doubles) {
  if (n_doubles != p->ndata) return DYNOHIP_EINVAL;
  memcpy(p->data, data, p->ndata * sizeof(double));
  p->error = graph_error(p, p->data);
  return 0;
}
int oracle_get_trace(const oracle_problem* p, dynohip_trace_entry* out, size_t cap, size_t* n_out) {
  const size_t n = p->ntrace < cap ? p->ntrace : cap;
  if (out && n) memcpy(out, p->trace, n * sizeof(dynohip_trace_entry));
  if (n_out) *n_out = p->ntrace;
  return 0;
}

/* ------------------------------------------------------------------ */
/* Threaded LM (oracle_set_threads): the all-cores CPU baseline.       */
/* Every parallel phase writes disjoint data; the sums that cross      */
/* threads are formed from per-factor / per-row terms added in the     */
/* serial order, and the envelope Cholesky subtracts its terms in the  */
/* serial order too, so the trajectory is bit-identical to the single- */
/* thread path.                                                        */
/* ------------------------------------------------------------------ */
typedef void (*task_fn)(void* ctx, int tid, int nt);
struct pool_t {
  int n;
  pthread_t* th;
  pthread_barrier_t start, end;
  task_fn fn;
  void* ctx;
  int quit;
};
typedef struct { struct pool_t* pool; int tid; } worker_arg;

static void* pool_worker(void* a) {
  worker_arg* w = (worker_arg*)a;
  struct pool_t* P = w->pool;
  const int tid = w->tid;
  free(w);
  for (;;) {
    pthread_barrier_wait(&P->start);
    if (P->quit) break;
    P->fn(P->ctx, tid, P->n);
    pthread_barrier_wait(&P->end);
  }
  return NULL;
}

static void pool_run(struct pool_t* P, task_fn fn, void* ctx) {
  P->fn = fn;
  P->ctx = ctx;
  pthread_barrier_wait(&P->start);
  fn(ctx, 0, P->n);
  pthread_barrier_wait(&P->end);
}

int oracle_set_threads(oracle_problem* p, int n) {
  if (!p) return DYNOHIP_EINVAL;
  if (p->pool) {
    struct pool_t* P = p->pool;
    P->quit = 1;
    pthread_barrier_wait(&P->start);
    for (int t = 1; t < P->n; ++t) pthread_join(P->th[t], NULL);
    pthread_barrier_destroy(&P->start);
    pthread_barrier_destroy(&P->end);
    free(P->th);
    free(P);
    p->pool = NULL;
  }
  p->nthreads = n > 1 ? n : 1;
  if (p->nthreads == 1) return 0;
  struct pool_t* P = (struct pool_t*)calloc(1, sizeof(struct pool_t));
  P->n = p->nthreads;
  P->th = (pthread_t*)calloc((size_t)P->n, sizeof(pthread_t));
  pthread_barrier_init(&P->start, NULL, (unsigned)P->n);
  pthread_barrier_init(&P->end, NULL, (unsigned)P->n);
  for (int t = 1; t < P->n; ++t) {
    worker_arg* w = (worker_arg*)malloc(sizeof(worker_arg));
    w->pool = P;
    w->tid = t;
    pthread_create(&P->th[t], NULL, pool_worker, w);
  }
  p->pool = P;
  /* factors touching each component (a factor's points share one) */
  if (!p->comp_f_start) {
    p->comp_f_start = (size_t*)calloc((size_t)p->ncomp + 1, sizeof(size_t));
    int* fc = (int*)malloc((p->nf ? p->nf : 1) * sizeof(int));
    for (size_t f = 0; f < p->nf; ++f) {
      const factor_t* F = &p->f[f];
      fc[f] = -1;
      for (int sl = 0; sl < kNKeys[F->type]; ++sl)
        if (kSlotKind[F->type][sl] == 1) fc[f] = p->comp_of[F->var[sl]];
      if (fc[f] >= 0) p->comp_f_start[fc[f] + 1]++;
    }
    for (int c = 0; c < p->ncomp; ++c) p->comp_f_start[c + 1] += p->comp_f_start[c];
    p->comp_f = (int*)malloc((p->comp_f_start[p->ncomp] ? p->comp_f_start[p->ncomp] : 1) * sizeof(int));
    size_t* fill = (size_t*)malloc(((size_t)p->ncomp + 1) * sizeof(size_t));
    memcpy(fill, p->comp_f_start, ((size_t)p->ncomp + 1) * sizeof(size_t));
    for (size_t f = 0; f < p->nf; ++f)
      if (fc[f] >= 0) p->comp_f[fill[fc[f]]++] = (int)f;
    free(fill);
    free(fc);
  }
  return 0;
}

static void chunk(size_t n, int tid, int nt, size_t* lo, size_t* hi) {
  *lo = n * (size_t)tid / (size_t)nt;
  *hi = n * (size_t)(tid + 1) / (size_t)nt;
}

typedef struct {
  oracle_problem* p;
  const double* data;
  const double* delta;
  const size_t* doff;
  double* terms;
  double lambda;
  int* tfail;
  size_t j0, j1, ilo, ihi;
} mt_ctx;

static void t_linearize(void* c, int tid, int nt) {
  mt_ctx* x = (mt_ctx*)c;
  size_t lo, hi;
  chunk(x->p->nf, tid, nt, &lo, &hi);
  for (size_t f = lo; f < hi; ++f) linearize_one(x->p, f);
}
static void linearize_all_mt(oracle_problem* p) {
  mt_ctx x;
  memset(&x, 0, sizeof(x));
  x.p = p;
  pool_run(p->pool, t_linearize, &x);
}

static void t_error(void* c, int tid, int nt) {
  mt_ctx* x = (mt_ctx*)c;
  size_t lo, hi;
  chunk(x->p->nf, tid, nt, &lo, &hi);
  for (size_t f = lo; f < hi; ++f) x->terms[f] = factor_error(x->p, x->data, &x->p->f[f]);
}
static double graph_error_mt(const oracle_problem* p, const double* data) {
  mt_ctx x;
  memset(&x, 0, sizeof(x));
  x.p = (oracle_problem*)p;
  x.data = data;
  x.terms = (double*)malloc((p->nf ? p->nf : 1) * sizeof(double));
  pool_run(p->pool, t_error, &x);
  double s = 0.0;
  for (size_t f = 0; f < p->nf; ++f) s += x.terms[f];
  free(x.terms);
  return s;
}

static void t_linerr(void* c, int tid, int nt) {
  mt_ctx* x = (mt_ctx*)c;
  size_t lo, hi;
  chunk(x->p->nf, tid, nt, &lo, &hi);
  for (size_t f = lo; f < hi; ++f) linear_error_rows(x->p, f, x->delta, x->doff, x->terms);
}
static double linear_error_mt(const oracle_problem* p, const double* delta, const size_t* doff) {
  size_t nrows = 0;
  for (size_t f = 0; f < p->nf; ++f) nrows += (size_t)kDim[p->f[f].type];
  mt_ctx x;
  memset(&x, 0, sizeof(x));
  x.p = (oracle_problem*)p;
  x.delta = delta;
  x.doff = doff;
  x.terms = (double*)malloc((nrows ? nrows : 1) * sizeof(double));
  pool_run(p->pool, t_linerr, &x);
  double s = 0.0;
  for (size_t r = 0; r < nrows; ++r) s += x.terms[r];
  free(x.terms);
  return 0.5 * s;
}

static int nb_index(const comp_t* C, int red) {
  int lo = 0, hi = C->nnb - 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (C->nb[mid] < red) lo = mid + 1; else hi = mid;
  }
  return lo;
}

/* zero the normal equations; each component's C, W, g_p from its own factors */
static void t_comp_accumulate(void* c, int tid, int nt) {
  mt_ctx* x = (mt_ctx*)c;
  oracle_problem* p = x->p;
  size_t lo, hi;
  chunk(p->rowoff[p->ndim_red], tid, nt, &lo, &hi);
  memset(p->sky + lo, 0, (hi - lo) * sizeof(double));
  chunk(p->ndim_red, tid, nt, &lo, &hi);
  memset(p->gc + lo, 0, (hi - lo) * sizeof(double));
  for (int cc = tid; cc < p->ncomp; cc += nt) {
    comp_t* C = &p->comps[cc];
    const size_t n3 = 3 * (size_t)C->npts, m6 = 6 * (size_t)C->nnb;
    memset(C->C, 0, n3 * n3 * sizeof(double));
    memset(C->W, 0, n3 * m6 * sizeof(double));
    memset(C->gp, 0, n3 * sizeof(double));
    for (size_t q = p->comp_f_start[cc]; q < p->comp_f_start[cc + 1]; ++q) {
      const size_t f = (size_t)p->comp_f[q];
      const factor_t* F = &p->f[f];
      const int d = kDim[F->type], cols = oracle_factor_cols(F->type), nk = kNKeys[F->type];
      const double* A = p->A + p->foffA[f];
      const double* b = p->b + p->foffb[f];
      int c0 = 0;
      for (int sa = 0; sa < nk; ++sa) {
        const int da = slot_dim(F->type, sa);
        if (kSlotKind[F->type][sa] != 1) { c0 += da; continue; }
        int la = 0;
        while (C->pts[la] != F->var[sa]) ++la;
        for (int ia = 0; ia < da; ++ia) {
          double s = 0.0;
          for (int r = 0; r < d; ++r) s += A[r * cols + c0 + ia] * b[r];
          C->gp[3 * la + ia] += s;
        }
        int c1 = 0;
        for (int sb = 0; sb < nk; ++sb) {
          const int db = slot_dim(F->type, sb);
          const int vb = F->var[sb];
          const int pb = kSlotKind[F->type][sb] == 1;
          size_t lb = 0;
          if (pb) { while (C->pts[lb] != vb) ++lb; }
          else lb = (size_t)nb_index(C, p->red_of[vb]);
          for (int ia = 0; ia < da; ++ia)
            for (int ib = 0; ib < db; ++ib) {
              double s = 0.0;
              for (int r = 0; r < d; ++r) s += A[r * cols + c0 + ia] * A[r * cols + c1 + ib];
              if (pb) C->C[(3 * (size_t)la + ia) * n3 + 3 * lb + ib] += s;
              else C->W[(3 * (size_t)la + ia) * m6 + 6 * lb + ib] += s;
            }
          c1 += db;
        }
        c0 += da;
      }
    }
  }
}

/* pose-side gradient and pose-pose blocks: thread t owns a range of
   reduced poses (rows), every thread scans the factors in order */
static void pose_range(const oracle_problem* p, int tid, int nt, int* lo, int* hi) {
  size_t a, b;
  chunk((size_t)p->npose, tid, nt, &a, &b);
  *lo = (int)a;
  *hi = (int)b;
}
static void t_pose_accumulate(void* c, int tid, int nt) {
  mt_ctx* x = (mt_ctx*)c;
  oracle_problem* p = x->p;
  int plo, phi;
  pose_range(p, tid, nt, &plo, &phi);
  for (size_t f = 0; f < p->nf; ++f) {
    const factor_t* F = &p->f[f];
    const int d = kDim[F->type], cols = oracle_factor_cols(F->type), nk = kNKeys[F->type];
    int mine = 0;
    for (int sa = 0; sa < nk; ++sa)
      if (kSlotKind[F->type][sa] == 0 && p->red_of[F->var[sa]] >= plo && p->red_of[F->var[sa]] < phi) mine = 1;
    if (!mine) continue;
    const double* A = p->A + p->foffA[f];
    const double* b = p->b + p->foffb[f];
    int c0 = 0;
    for (int sa = 0; sa < nk; ++sa) {
      const int da = slot_dim(F->type, sa);
      const int va = F->var[sa];
      if (kSlotKind[F->type][sa] != 0 || p->red_of[va] < plo || p->red_of[va] >= phi) { c0 += da; continue; }
      for (int ia = 0; ia < da; ++ia) {
        double s = 0.0;
        for (int r = 0; r < d; ++r) s += A[r * cols + c0 + ia] * b[r];
        p->gc[6 * (size_t)p->red_of[va] + ia] += s;
      }
      int c1 = 0;
      for (int sb = 0; sb < nk; ++sb) {
        const int db = slot_dim(F->type, sb);
        const int vb = F->var[sb];
        if (kSlotKind[F->type][sb] == 0)
          for (int ia = 0; ia < da; ++ia)
            for (int ib = 0; ib < db; ++ib) {
              const size_t gi = 6 * (size_t)p->red_of[va] + ia, gj = 6 * (size_t)p->red_of[vb] + ib;
              if (gi < gj) continue;
              double s = 0.0;
              for (int r = 0; r < d; ++r) s += A[r * cols + c0 + ia] * A[r * cols + c1 + ib];
              *sky_at(p, gi, gj) += s;
            }
        c1 += db;
      }
      c0 += da;
    }
  }
  for (size_t i = 6 * (size_t)plo; i < 6 * (size_t)phi; ++i) *sky_at(p, i, i) += x->lambda;
}

static void t_comp_factor(void* c, int tid, int nt) {
  mt_ctx* x = (mt_ctx*)c;
  oracle_problem* p = x->p;
  for (int cc = tid; cc < p->ncomp; cc += nt) {
    comp_t* C = &p->comps[cc];
    const size_t n3 = 3 * (size_t)C->npts, m6 = 6 * (size_t)C->nnb;
    for (size_t i = 0; i < n3; ++i) C->C[i * n3 + i] += x->lambda;
    if (!chol_dense(C->C, n3)) { x->tfail[tid] = 1; continue; }
    memcpy(C->Y, C->W, n3 * m6 * sizeof(double));
    chol_solve(C->C, n3, C->Y, m6);
    memcpy(C->v, C->gp, n3 * sizeof(double));
    chol_solve(C->C, n3, C->v, 1);
  }
}

/* Schur terms into the rows this thread owns, components in order */
static void t_schur(void* c, int tid, int nt) {
  mt_ctx* x = (mt_ctx*)c;
  oracle_problem* p = x->p;
  int plo, phi;
  pose_range(p, tid, nt, &plo, &phi);
  for (int cc = 0; cc < p->ncomp; ++cc) {
    comp_t* C = &p->comps[cc];
    const size_t n3 = 3 * (size_t)C->npts, m6 = 6 * (size_t)C->nnb;
    for (int a = 0; a < C->nnb; ++a) {
      if (C->nb[a] < plo || C->nb[a] >= phi) continue;
      for (int ia = 0; ia < 6; ++ia) {
        const size_t gi = 6 * (size_t)C->nb[a] + ia;
        double s = 0.0;
        for (size_t k = 0; k < n3; ++k) s += C->W[k * m6 + 6 * a + ia] * C->v[k];
        p->gc[gi] -= s;
        for (int bb = 0; bb <= a; ++bb)
          for (int ib = 0; ib < 6; ++ib) {
            const size_t gj = 6 * (size_t)C->nb[bb] + ib;
            if (gj > gi) continue;
            double t = 0.0;
            for (size_t k = 0; k < n3; ++k) t += C->W[k * m6 + 6 * a + ia] * C->Y[k * m6 + 6 * bb + ib];
            *sky_at(p, gi, gj) -= t;
          }
      }
    }
  }
}

/* blocked right-looking envelope Cholesky, rows [ilo, ihi) of block [j0, j1):
   panel entries (columns of the block), then the trailing update; the terms
   of every entry are subtracted in ascending k, as the serial row form does */
static void t_chol_panel(void* c, int tid, int nt) {
  mt_ctx* x = (mt_ctx*)c;
  oracle_problem* p = x->p;
  for (size_t i = x->ilo + (size_t)tid; i < x->ihi; i += (size_t)nt) {
    const size_t fi = p->first[i];
    if (fi >= x->j1) continue;
    for (size_t j = fi > x->j0 ? fi : x->j0; j < x->j1; ++j) {
      const size_t fj = p->first[j];
      size_t k0 = fi > fj ? fi : fj;
      if (k0 < x->j0) k0 = x->j0;
      double s = *sky_at(p, i, j);
      for (size_t k = k0; k < j; ++k) s -= *sky_at(p, i, k) * *sky_at(p, j, k);
      *sky_at(p, i, j) = s / *sky_at(p, j, j);
    }
  }
}
static void t_chol_update(void* c, int tid, int nt) {
  mt_ctx* x = (mt_ctx*)c;
  oracle_problem* p = x->p;
  for (size_t i = x->ilo + (size_t)tid; i < x->ihi; i += (size_t)nt) {
    const size_t fi = p->first[i];
    if (fi >= x->j1) continue;
    for (size_t j = fi > x->j1 ? fi : x->j1; j <= i; ++j) {
      const size_t fj = p->first[j];
      if (fj >= x->j1) continue;
      size_t k0 = fi > fj ? fi : fj;
      if (k0 < x->j0) k0 = x->j0;
      double s = *sky_at(p, i, j);
      for (size_t k = k0; k < x->j1; ++k) s -= *sky_at(p, i, k) * *sky_at(p, j, k);
      *sky_at(p, i, j) = s;
    }
  }
}

static void t_backsub(void* c, int tid, int nt) {
  mt_ctx* x = (mt_ctx*)c;
  oracle_problem* p = x->p;
  double* delta = (double*)x->delta;
  for (int cc = tid; cc < p->ncomp; cc += nt) {
    comp_t* C = &p->comps[cc];
    const size_t n3 = 3 * (size_t)C->npts, m6 = 6 * (size_t)C->nnb;
    double* rhs = (double*)malloc((n3 ? n3 : 1) * sizeof(double));
    for (size_t k = 0; k < n3; ++k) {
      double s = C->gp[k];
      for (int a = 0; a < C->nnb; ++a)
        for (int ia = 0; ia < 6; ++ia)
          s -= C->W[k * m6 + 6 * a + ia] * delta[x->doff[p->pose_var[C->nb[a]]] + ia];
      rhs[k] = s;
    }
    chol_solve(C->C, n3, rhs, 1);
    for (int k = 0; k < C->npts; ++k)
      for (int j = 0; j < 3; ++j) delta[x->doff[C->pts[k]] + j] = rhs[3 * k + j];
    free(rhs);
  }
}

static int solve_schur_mt(oracle_problem* p, double lambda, double* delta, const size_t* doff) {
  const size_t nd = p->ndim_red;
  const int nt = p->nthreads;
  mt_ctx x;
  memset(&x, 0, sizeof(x));
  x.p = p;
  x.lambda = lambda;
  x.doff = doff;
  x.delta = delta;
  x.tfail = (int*)calloc((size_t)nt, sizeof(int));
  pool_run(p->pool, t_comp_accumulate, &x);
  pool_run(p->pool, t_pose_accumulate, &x);
  pool_run(p->pool, t_comp_factor, &x);
  int ok = 1;
  for (int t = 0; t < nt; ++t) ok = ok && !x.tfail[t];
  free(x.tfail);
  if (!ok) return 0;
  pool_run(p->pool, t_schur, &x);
  /* envelope Cholesky, 64-column blocks */
  const size_t B = 64;
  for (size_t j0 = 0; j0 < nd; j0 += B) {
    const size_t j1 = j0 + B < nd ? j0 + B : nd;
    /* the diagonal block, serially (its rows, its columns) */
    for (size_t i = j0; i < j1; ++i) {
      const size_t fi = p->first[i];
      for (size_t j = fi > j0 ? fi : j0; j <= i; ++j) {
        const size_t fj = p->first[j];
        size_t k0 = fi > fj ? fi : fj;
        if (k0 < j0) k0 = j0;
        double s = *sky_at(p, i, j);
        for (size_t k = k0; k < j; ++k) s -= *sky_at(p, i, k) * *sky_at(p, j, k);
        if (j == i) {
          if (!(s > 0.0) || !isfinite(s)) return 0;
          *sky_at(p, i, i) = sqrt(s);
        } else {
          *sky_at(p, i, j) = s / *sky_at(p, j, j);
        }
      }
    }
    size_t ihi = j1;
    for (size_t i = j1; i < nd; ++i)
      if (p->first[i] < j1) ihi = i + 1;
    if (ihi > j1) {
      x.j0 = j0;
      x.j1 = j1;
      x.ilo = j1;
      x.ihi = ihi;
      pool_run(p->pool, t_chol_panel, &x);
      pool_run(p->pool, t_chol_update, &x);
    }
  }
  /* forward / backward substitution */
  double* y = (double*)malloc((nd ? nd : 1) * sizeof(double));
  for (size_t i = 0; i < nd; ++i) {
    double s = p->gc[i];
    for (size_t k = p->first[i]; k < i; ++k) s -= *sky_at(p, i, k) * y[k];
    y[i] = s / *sky_at(p, i, i);
  }
  for (size_t ii = nd; ii-- > 0;) {
    y[ii] /= *sky_at(p, ii, ii);
    const double xi = y[ii];
    for (size_t k = p->first[ii]; k < ii; ++k) y[k] -= *sky_at(p, ii, k) * xi;
  }
  for (int r = 0; r < p->npose; ++r)
    for (int k = 0; k < 6; ++k) delta[doff[p->pose_var[r]] + k] = y[6 * (size_t)r + k];
  free(y);
  pool_run(p->pool, t_backsub, &x);
  return 1;
}
