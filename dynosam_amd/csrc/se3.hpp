// se3.hpp — FP64 SO(3)/SE(3) for device (and host) code.
//
// Semantics of GTSAM 4.2.0 with GTSAM_POSE3_EXPMAP / GTSAM_ROT3_EXPMAP
// (docker/Dockerfile:88): Rot3 stored as a 3x3 matrix, retract T·Exp(ξ),
// ξ = [ω; v]. Poses are 12 doubles: R row-major then t.
#pragma once

#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>

// No fused multiply-add contraction in the pose arithmetic: every product
// and sum is rounded as the CPU restatement rounds it (oracle/oracle.c, the
// same formulas in the same order, compiled without FMA), so the residuals
// and Jacobians of the factor kernels are bit-identical to the oracle's.
// Near convergence the Huber weights k/||r|| of the sigma-1e-5 ternary
// factors are computed from residuals dominated by cancellation; rounding
// them differently moved whole Jacobian rows by ~1e-5.
#pragma clang fp contract(off)

// sin, tan and acos shared with the CPU oracle (identical rounding)
#include "trig.h"

namespace dynohip {

#define DH_HD __host__ __device__ __forceinline__

struct P3 {
  double R[9];
  double t[3];
};

DH_HD void load_pose(const double* __restrict__ p, P3& T) {
#pragma unroll
  for (int i = 0; i < 9; ++i) T.R[i] = p[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) T.t[i] = p[9 + i];
}

DH_HD void store_pose(double* __restrict__ p, const P3& T) {
#pragma unroll
  for (int i = 0; i < 9; ++i) p[i] = T.R[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) p[9 + i] = T.t[i];
}

DH_HD void mat3_mul(const double* A, const double* B, double* C) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      C[3 * i + j] = A[3 * i + 0] * B[0 + j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

DH_HD void mat3_vec(const double* A, const double* v, double* o) {
#pragma unroll
  for (int i = 0; i < 3; ++i) o[i] = A[3 * i] * v[0] + A[3 * i + 1] * v[1] + A[3 * i + 2] * v[2];
}

DH_HD void mat3t_vec(const double* A, const double* v, double* o) {
#pragma unroll
  for (int i = 0; i < 3; ++i) o[i] = A[i] * v[0] + A[3 + i] * v[1] + A[6 + i] * v[2];
}

DH_HD P3 compose(const P3& A, const P3& B) {
  P3 C;
  mat3_mul(A.R, B.R, C.R);
  mat3_vec(A.R, B.t, C.t);
#pragma unroll
  for (int i = 0; i < 3; ++i) C.t[i] += A.t[i];
  return C;
}

DH_HD P3 inverse(const P3& A) {
  P3 C;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) C.R[3 * i + j] = A.R[3 * j + i];
  double t[3];
  mat3_vec(C.R, A.t, t);
  C.t[0] = -t[0];
  C.t[1] = -t[1];
  C.t[2] = -t[2];
  return C;
}

// Pose3::transformFrom: R p + t
DH_HD void transform_from(const P3& T, const double* p, double* o) {
  double q[3];
  mat3_vec(T.R, p, q);
  o[0] = q[0] + T.t[0];
  o[1] = q[1] + T.t[1];
  o[2] = q[2] + T.t[2];
}

// so3::ExpmapFunctor::expmap
DH_HD void rot_expmap(const double* w, double* R) {
  const double theta2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  const double W[9] = {0.0, -w[2], w[1], w[2], 0.0, -w[0], -w[1], w[0], 0.0};
  if (theta2 <= DBL_EPSILON) {
#pragma unroll
    for (int i = 0; i < 9; ++i) R[i] = W[i];
    R[0] += 1.0;
    R[4] += 1.0;
    R[8] += 1.0;
    return;
  }
  const double theta = sqrt(theta2);
  double K[9], KK[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) K[i] = W[i] / theta;
  mat3_mul(K, K, KK);
  const double s = dht_sin(theta);
  const double s2 = dht_sin(theta / 2.0);
  const double omc = 2.0 * s2 * s2;
#pragma unroll
  for (int i = 0; i < 9; ++i) R[i] = s * K[i] + omc * KK[i];
  R[0] += 1.0;
  R[4] += 1.0;
  R[8] += 1.0;
}

// SO3::Logmap (GTSAM 4.2.0)
DH_HD void rot_logmap(const double* R, double* w) {
  const double R11 = R[0], R12 = R[1], R13 = R[2];
  const double R21 = R[3], R22 = R[4], R23 = R[5];
  const double R31 = R[6], R32 = R[7], R33 = R[8];
  const double tr = R11 + R22 + R33;
  if (tr + 1.0 < 1e-3) {
    double Wv, Q1, Q2, Q3;
    int which;
    if (R33 > R22 && R33 > R11) {
      Wv = R21 - R12; Q1 = 2.0 + 2.0 * R33; Q2 = R31 + R13; Q3 = R23 + R32; which = 3;
    } else if (R22 > R11) {
      Wv = R13 - R31; Q1 = 2.0 + 2.0 * R22; Q2 = R23 + R32; Q3 = R12 + R21; which = 2;
    } else {
      Wv = R32 - R23; Q1 = 2.0 + 2.0 * R11; Q2 = R12 + R21; Q3 = R31 + R13; which = 1;
    }
    const double r = sqrt(Q1);
    const double one_over_r = 1 / r;
    const double norm = sqrt(Q1 * Q1 + Q2 * Q2 + Q3 * Q3 + Wv * Wv);
    const double sgn_w = Wv < 0 ? -1.0 : 1.0;
    const double mag = M_PI - (2 * sgn_w * Wv) / norm;
    const double scale = 0.5 * one_over_r * mag;
    if (which == 3) { w[0] = sgn_w * scale * Q2; w[1] = sgn_w * scale * Q3; w[2] = sgn_w * scale * Q1; }
    else if (which == 2) { w[0] = sgn_w * scale * Q3; w[1] = sgn_w * scale * Q1; w[2] = sgn_w * scale * Q2; }
    else { w[0] = sgn_w * scale * Q1; w[1] = sgn_w * scale * Q2; w[2] = sgn_w * scale * Q3; }
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

// Pose3::Expmap
DH_HD P3 pose_expmap(const double* xi) {
  P3 T;
  const double* w = xi;
  const double* v = xi + 3;
  rot_expmap(w, T.R);
  const double theta2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  if (theta2 > DBL_EPSILON) {
    const double wv = w[0] * v[0] + w[1] * v[1] + w[2] * v[2];
    const double wxv[3] = {w[1] * v[2] - w[2] * v[1], w[2] * v[0] - w[0] * v[2], w[0] * v[1] - w[1] * v[0]};
    double Rwxv[3];
    mat3_vec(T.R, wxv, Rwxv);
#pragma unroll
    for (int i = 0; i < 3; ++i) T.t[i] = (wxv[i] - Rwxv[i] + w[i] * wv) / theta2;
  } else {
    T.t[0] = v[0];
    T.t[1] = v[1];
    T.t[2] = v[2];
  }
  return T;
}

// Pose3::Logmap
DH_HD void pose_logmap(const P3& T, double* xi) {
  double w[3];
  rot_logmap(T.R, w);
  const double th = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  xi[0] = w[0];
  xi[1] = w[1];
  xi[2] = w[2];
  if (th < 1e-10) {
    xi[3] = T.t[0];
    xi[4] = T.t[1];
    xi[5] = T.t[2];
    return;
  }
  const double wn[3] = {w[0] / th, w[1] / th, w[2] / th};
  const double W[9] = {0.0, -wn[2], wn[1], wn[2], 0.0, -wn[0], -wn[1], wn[0], 0.0};
  const double Tan = dht_tan(0.5 * th);
  double WT[3], WWT[3];
  mat3_vec(W, T.t, WT);
  mat3_vec(W, WT, WWT);
  const double c = 1 - th / (2. * Tan);
#pragma unroll
  for (int i = 0; i < 3; ++i) xi[3 + i] = T.t[i] - (0.5 * th) * WT[i] + c * WWT[i];
}

DH_HD P3 pose_retract(const P3& T, const double* xi) { return compose(T, pose_expmap(xi)); }

}  // namespace dynohip

#pragma clang fp contract(fast)
