// refine.hip — batched object-motion refinement on the GPU (SURVEY.md §8(f)
// row 4, include/dynorefine.h): MotionOnlyRefinementOptimizer::optimize with
// the ProjectionError solver (dynosam/include/dynosam/frontend/vision/
// MotionSolver-inl.hpp:277-470) for thousands of (object, frame pair)
// problems in one launch.
//
// Per problem: priors on X_{k-1}, X_k, the object motion H and, per
// tracklet, the points m_{k-1}, m_k with two GenericProjectionFactor
// <Pose3, Point3, Cal3_S2> and one LandmarkMotionTernaryFactor; GTSAM 4.2
// LevenbergMarquardtOptimizer semantics (default parameters) — the same
// decisions as the backend solver (solver.cpp lm_iterate) and the checker
// oracle/refine.py.
//
// Mapping: one 64-wide wavefront per problem; lanes own tracklets (chunks of
// 64). The damped normal equations are solved through the Schur complement
// of every tracklet's 6x6 point block: a lane factors its C_i + lambda I in
// registers, forms Y_i = C_i^-1 W_i, and the wave sums B_i - W_i^T Y_i into
// the 18x18 (X_{k-1}, X_k, H) system through an LDS transpose (64 entries at
// a time, each summed by one lane in lane order: bit-reproducible). The
// 18x18 system is factored in registers (lane = row, readlane broadcasts),
// then every lane back-substitutes its points. The whole LM loop (linearise, tryLambda,
// accept / reject, convergence, outlier rounds) runs inside the kernel: one
// launch per batch, no host round trip per iteration.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cstdio>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/dynorefine.h"

namespace {

constexpr int kWave = 64;
constexpr int kLin = 80;  // linearisation scratch per tracklet (doubles)
constexpr int kWin = 63;  // reduction window: 57 system entries + 6 gradient entries
constexpr int kQuads = kWave / 4;  // reduction columns: quad sums
constexpr int kRedLd = kQuads + 1;
constexpr double kChi2_3_099 = 11.344866730144373;  // boost chi_squared quantile(3, 0.99)

struct Pose {
  double R[9];
  double t[3];
};

__device__ __forceinline__ void load_pose(const double* p, Pose& T) {
#pragma unroll
  for (int i = 0; i < 9; ++i) T.R[i] = p[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) T.t[i] = p[9 + i];
}
__device__ __forceinline__ void store_pose(double* p, const Pose& T) {
#pragma unroll
  for (int i = 0; i < 9; ++i) p[i] = T.R[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) p[9 + i] = T.t[i];
}

// ---- SO(3) / SE(3), GTSAM 4.2 with EXPMAP (as csrc/se3.hpp) ----
__device__ void rot_expmap(const double* w, double* R) {
  const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  const double W[9] = {0.0, -w[2], w[1], w[2], 0.0, -w[0], -w[1], w[0], 0.0};
  if (th2 <= DBL_EPSILON) {
    for (int i = 0; i < 9; ++i) R[i] = W[i] + ((i % 4) == 0 ? 1.0 : 0.0);
    return;
  }
  const double th = sqrt(th2);
  double K[9], KK[9];
  for (int i = 0; i < 9; ++i) K[i] = W[i] / th;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) KK[3 * i + j] = K[3 * i] * K[j] + K[3 * i + 1] * K[3 + j] + K[3 * i + 2] * K[6 + j];
  const double s = sin(th), s2 = sin(th / 2.0), c1 = 2.0 * s2 * s2;
  for (int i = 0; i < 9; ++i) R[i] = ((i % 4) == 0 ? 1.0 : 0.0) + s * K[i] + c1 * KK[i];
}

__device__ void rot_logmap(const double* R, double* w) {
  const double R11 = R[0], R12 = R[1], R13 = R[2], R21 = R[3], R22 = R[4], R23 = R[5], R31 = R[6], R32 = R[7],
               R33 = R[8];
  const double tr = R11 + R22 + R33;
  if (tr + 1.0 < 1e-3) {
    double W, Q1, Q2, Q3;
    int which;
    if (R33 > R22 && R33 > R11) {
      W = R21 - R12; Q1 = 2.0 + 2.0 * R33; Q2 = R31 + R13; Q3 = R23 + R32; which = 3;
    } else if (R22 > R11) {
      W = R13 - R31; Q1 = 2.0 + 2.0 * R22; Q2 = R23 + R32; Q3 = R12 + R21; which = 2;
    } else {
      W = R32 - R23; Q1 = 2.0 + 2.0 * R11; Q2 = R12 + R21; Q3 = R31 + R13; which = 1;
    }
    const double r = sqrt(Q1);
    const double norm = sqrt(Q1 * Q1 + Q2 * Q2 + Q3 * Q3 + W * W);
    const double sgn = W < 0 ? -1.0 : 1.0;
    const double mag = M_PI - (2 * sgn * W) / norm;
    const double sc = sgn * (0.5 * (1 / r) * mag);
    if (which == 3) { w[0] = sc * Q2; w[1] = sc * Q3; w[2] = sc * Q1; }
    else if (which == 2) { w[0] = sc * Q3; w[1] = sc * Q1; w[2] = sc * Q2; }
    else { w[0] = sc * Q1; w[1] = sc * Q2; w[2] = sc * Q3; }
    return;
  }
  const double tr_3 = tr - 3.0;
  double m;
  if (tr_3 < -1e-6) {
    const double th = acos((tr - 1.0) / 2.0);
    m = th / (2.0 * sin(th));
  } else {
    m = 0.5 - tr_3 / 12.0 + tr_3 * tr_3 / 60.0;
  }
  w[0] = m * (R32 - R23);
  w[1] = m * (R13 - R31);
  w[2] = m * (R21 - R12);
}

// T * Expmap(xi)
__device__ void pose_retract(const Pose& T, const double* xi, Pose& out) {
  double dR[9], dt[3];
  const double* w = xi;
  const double* v = xi + 3;
  rot_expmap(w, dR);
  const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  if (th2 > DBL_EPSILON) {
    const double wv = w[0] * v[0] + w[1] * v[1] + w[2] * v[2];
    const double wxv[3] = {w[1] * v[2] - w[2] * v[1], w[2] * v[0] - w[0] * v[2], w[0] * v[1] - w[1] * v[0]};
    for (int i = 0; i < 3; ++i) {
      const double Rw = dR[3 * i] * wxv[0] + dR[3 * i + 1] * wxv[1] + dR[3 * i + 2] * wxv[2];
      dt[i] = (wxv[i] - Rw + w[i] * wv) / th2;
    }
  } else {
    dt[0] = v[0]; dt[1] = v[1]; dt[2] = v[2];
  }
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j)
      out.R[3 * i + j] = T.R[3 * i] * dR[j] + T.R[3 * i + 1] * dR[3 + j] + T.R[3 * i + 2] * dR[6 + j];
    out.t[i] = T.R[3 * i] * dt[0] + T.R[3 * i + 1] * dt[1] + T.R[3 * i + 2] * dt[2] + T.t[i];
  }
}

// PriorFactor<Pose3>::evaluateError: r = -Logmap(X^-1 Z) (H = I)
__device__ void prior_residual(const Pose& X, const Pose& Z, double* r) {
  Pose e;
  const double d[3] = {Z.t[0] - X.t[0], Z.t[1] - X.t[1], Z.t[2] - X.t[2]};
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j)
      e.R[3 * i + j] = X.R[i] * Z.R[j] + X.R[3 + i] * Z.R[3 + j] + X.R[6 + i] * Z.R[6 + j];
    e.t[i] = X.R[i] * d[0] + X.R[3 + i] * d[1] + X.R[6 + i] * d[2];
  }
  double w[3];
  rot_logmap(e.R, w);
  const double th = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  double u[3] = {e.t[0], e.t[1], e.t[2]};
  if (th >= 1e-10) {
    const double wn[3] = {w[0] / th, w[1] / th, w[2] / th};
    const double WT[3] = {wn[1] * e.t[2] - wn[2] * e.t[1], wn[2] * e.t[0] - wn[0] * e.t[2],
                          wn[0] * e.t[1] - wn[1] * e.t[0]};
    const double WWT[3] = {wn[1] * WT[2] - wn[2] * WT[1], wn[2] * WT[0] - wn[0] * WT[2],
                           wn[0] * WT[1] - wn[1] * WT[0]};
    const double c = 1 - th / (2. * tan(0.5 * th));
    for (int i = 0; i < 3; ++i) u[i] = e.t[i] - (0.5 * th) * WT[i] + c * WWT[i];
  }
  r[0] = -w[0]; r[1] = -w[1]; r[2] = -w[2];
  r[3] = -u[0]; r[4] = -u[1]; r[5] = -u[2];
}

__device__ __forceinline__ double huber_w(double e, double k) { return e <= k ? 1.0 : k / e; }
__device__ __forceinline__ double huber_rho(double e, double k) { return e <= k ? 0.5 * e * e : k * (e - 0.5 * k); }

// GenericProjectionFactor<Pose3, Point3, Cal3_S2> (throwCheirality = false).
// Returns the robust error; if A: whitened + Huber-reweighted
// A = [Jpose (6) | Jpoint (3)] (2x9 row-major) and b = -r.
__device__ double projection(const Pose& X, const double* p, const double* K, const double* kp, double isig,
                             double hk, double* A, double* b) {
  const double d0 = p[0] - X.t[0], d1 = p[1] - X.t[1], d2 = p[2] - X.t[2];
  const double q[3] = {X.R[0] * d0 + X.R[3] * d1 + X.R[6] * d2, X.R[1] * d0 + X.R[4] * d1 + X.R[7] * d2,
                       X.R[2] * d0 + X.R[5] * d1 + X.R[8] * d2};
  const double fx = K[0], fy = K[1], s = K[2], u0 = K[3], v0 = K[4];
  if (q[2] <= 0) {  // CheiralityException caught: (2 fx, 2 fx) and zero Jacobians
    const double rw = 2.0 * fx * isig;
    const double e = sqrt(rw * rw + rw * rw);
    if (A) {
      const double w = sqrt(huber_w(e, hk));
      for (int i = 0; i < 18; ++i) A[i] = 0.0;
      b[0] = b[1] = -rw * w;
    }
    return huber_rho(e, hk);
  }
  const double d = 1.0 / q[2];
  const double u = q[0] * d, v = q[1] * d;
  const double rw0 = (fx * u + s * v + u0 - kp[0]) * isig, rw1 = (fy * v + v0 - kp[1]) * isig;
  const double e = sqrt(rw0 * rw0 + rw1 * rw1);
  if (A) {
    const double w = sqrt(huber_w(e, hk));
    // PinholeBase::Dpose and Dpoint, then Cal3_S2 Dcal = [[fx, s], [0, fy]]
    const double P0[6] = {u * v, -(1 + u * u), v, -d, 0.0, d * u};
    const double P1[6] = {1 + v * v, -u * v, -u, 0.0, -d, d * v};
    double Q0[3], Q1[3];
    for (int j = 0; j < 3; ++j) {  // d [1, 0, -u] R^T and d [0, 1, -v] R^T
      Q0[j] = d * (X.R[3 * j + 0] - u * X.R[3 * j + 2]);
      Q1[j] = d * (X.R[3 * j + 1] - v * X.R[3 * j + 2]);
    }
    const double a0 = fx * isig * w, a1 = s * isig * w, a2 = fy * isig * w;
    for (int j = 0; j < 6; ++j) {
      A[j] = a0 * P0[j] + a1 * P1[j];
      A[9 + j] = a2 * P1[j];
    }
    for (int j = 0; j < 3; ++j) {
      A[6 + j] = a0 * Q0[j] + a1 * Q1[j];
      A[15 + j] = a2 * Q1[j];
    }
    b[0] = -rw0 * w;
    b[1] = -rw1 * w;
  }
  return huber_rho(e, hk);
}

// LandmarkMotionTernaryFactor (LandmarkMotionTernaryFactor.cc:37-73):
// r = m_{k-1} - H^-1 m_k. Returns the robust error; if A: whitened +
// reweighted A = [J1 (3) | J2 (3) | J3 (6)] (3x12), b = -r. *gauss = the
// Gaussian error 0.5 |r / sigma|^2 (determineFactorOutliers).
__device__ double ternary(const double* p1, const double* p2, const Pose& H, double isig, double hk, double* A,
                          double* b, double* gauss = nullptr) {
  const double d0 = p2[0] - H.t[0], d1 = p2[1] - H.t[1], d2 = p2[2] - H.t[2];
  const double q[3] = {H.R[0] * d0 + H.R[3] * d1 + H.R[6] * d2, H.R[1] * d0 + H.R[4] * d1 + H.R[7] * d2,
                       H.R[2] * d0 + H.R[5] * d1 + H.R[8] * d2};
  const double rw[3] = {(p1[0] - q[0]) * isig, (p1[1] - q[1]) * isig, (p1[2] - q[2]) * isig};
  const double e = sqrt(rw[0] * rw[0] + rw[1] * rw[1] + rw[2] * rw[2]);
  if (gauss) *gauss = 0.5 * e * e;
  if (A) {
    const double w = sqrt(huber_w(e, hk));
    const double sw = isig * w;
    for (int i = 0; i < 3; ++i) {
      double* row = A + 12 * i;
      for (int j = 0; j < 3; ++j) {
        row[j] = (i == j) ? sw : 0.0;       // J1 = I
        row[3 + j] = -H.R[3 * j + i] * sw;  // J2 = -R^T
        row[9 + j] = (i == j) ? sw : 0.0;   // J3, translation part = I
      }
      b[i] = -rw[i] * w;
    }
    // J3, rotation part = -skew(q)
    A[6] = 0.0;        A[7] = q[2] * sw;   A[8] = -q[1] * sw;
    A[18] = -q[2] * sw; A[19] = 0.0;       A[20] = q[0] * sw;
    A[30] = q[1] * sw;  A[31] = -q[0] * sw; A[32] = 0.0;
  }
  return huber_rho(e, hk);
}

// lane `src`'s v (src wave-uniform), through two v_readlane_b32
__device__ __forceinline__ double read_lane(double v, int src) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane(static_cast<unsigned>(u), src);
  const unsigned hi = __builtin_amdgcn_readlane(static_cast<unsigned>(u >> 32), src);
  return __longlong_as_double((static_cast<unsigned long long>(hi) << 32) | lo);
}

// v from the lane given by the DPP quad permutation CTRL
template <int CTRL>
__device__ __forceinline__ double quad_perm(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_mov_dpp(static_cast<int>(u), CTRL, 0xF, 0xF, false);
  const unsigned hi = __builtin_amdgcn_mov_dpp(static_cast<int>(u >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double((static_cast<unsigned long long>(hi) << 32) | lo);
}
// (v0 + v1) + (v2 + v3) over the lane's quad, identical on its four lanes
__device__ __forceinline__ double quad_sum(double v) {
  v += quad_perm<0xB1>(v);     // [1, 0, 3, 2]
  return v + quad_perm<0x4E>(v);  // [2, 3, 0, 1]
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// ---- per-tracklet Schur pieces from the linearisation scratch L ----
//   L[0:18]  A1 = [Jx | Jp] of the projection at k-1 (2x9), L[18:20] b1
//   L[20:38] A2 (projection at k),                          L[38:40] b2
//   L[40:76] At = [J1 | J2 | J3] (3x12),  L[76:79] bt,  L[79] 1 if the ternary is present

// C = point block (6x6) + lambda I, Cholesky-factored in place (lower)
__device__ bool point_block(const double* L, double lambda, double* C) {
  const double* A1 = L;
  const double* A2 = L + 20;
  const double* At = L + 40;
  const bool tern = L[79] != 0.0;
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = 0.0;
      if (i < 3 && j < 3) s += A1[6 + i] * A1[6 + j] + A1[15 + i] * A1[15 + j];
      if (i >= 3 && j >= 3) s += A2[3 + i] * A2[3 + j] + A2[12 + i] * A2[12 + j];
      if (tern) s += At[i] * At[j] + At[12 + i] * At[12 + j] + At[24 + i] * At[24 + j];
      if (i == j) s += lambda;
      C[6 * i + j] = s;
    }
  for (int k = 0; k < 6; ++k) {
    double d = C[7 * k];
    for (int m = 0; m < k; ++m) d -= C[6 * k + m] * C[6 * k + m];
    if (!(d > 0.0)) return false;
    d = sqrt(d);
    C[7 * k] = d;
    for (int i = k + 1; i < 6; ++i) {
      double s = C[6 * i + k];
      for (int m = 0; m < k; ++m) s -= C[6 * i + m] * C[6 * k + m];
      C[6 * i + k] = s / d;
    }
  }
  return true;
}

__device__ __forceinline__ void point_solve(const double* C, double* x) {
  for (int i = 0; i < 6; ++i) {
    double s = x[i];
    for (int m = 0; m < i; ++m) s -= C[6 * i + m] * x[m];
    x[i] = s / C[7 * i];
  }
  for (int i = 5; i >= 0; --i) {
    double s = x[i];
    for (int m = i + 1; m < 6; ++m) s -= C[6 * m + i] * x[m];
    x[i] = s / C[7 * i];
  }
}

// x <- L^-1 x (the forward half of point_solve)
__device__ __forceinline__ void lower_solve(const double* C, double* x) {
  for (int i = 0; i < 6; ++i) {
    double s = x[i];
    for (int m = 0; m < i; ++m) s -= C[6 * i + m] * x[m];
    x[i] = s / C[7 * i];
  }
}
__device__ __forceinline__ double dot6(const double* a, const double* b) {
  return ((a[0] * b[0] + a[1] * b[1]) + (a[2] * b[2] + a[3] * b[3])) + (a[4] * b[4] + a[5] * b[5]);
}
__device__ __forceinline__ double dot3(const double* a, const double* b) {
  return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2];
}

// W(:, c): point rows (6) of pose column c in [X1 (0-5) | X2 (6-11) | H (12-17)]
__device__ __forceinline__ void w_column(const double* L, int c, double* w) {
  const double* A1 = L;
  const double* A2 = L + 20;
  const double* At = L + 40;
  for (int i = 0; i < 6; ++i) w[i] = 0.0;
  if (c < 6) {
    for (int i = 0; i < 3; ++i) w[i] = A1[6 + i] * A1[c] + A1[15 + i] * A1[9 + c];
  } else if (c < 12) {
    for (int i = 0; i < 3; ++i) w[3 + i] = A2[6 + i] * A2[c - 6] + A2[15 + i] * A2[c + 3];
  } else if (L[79] != 0.0) {
    for (int i = 0; i < 6; ++i)
      w[i] = At[i] * At[c - 6] + At[12 + i] * At[c + 6] + At[24 + i] * At[c + 18];
  }
}
// z = L^-1 W(:, c); z_column_bot: rows 3-5 of z for an X_k column (c in
// 6-11), whose rows 0-2 are zero
__device__ __forceinline__ void z_column(const double* L, const double* C, int c, double* z) {
  w_column(L, c, z);
  lower_solve(C, z);
}
__device__ __forceinline__ void z_column_bot(const double* L, const double* C, int c, double* z) {
  const double* A2 = L + 20;
  for (int i = 0; i < 3; ++i) {
    double s = A2[6 + i] * A2[c - 6] + A2[15 + i] * A2[c + 3];
    for (int m = 0; m < i; ++m) s -= C[6 * (3 + i) + 3 + m] * z[m];
    z[i] = s / C[7 * (3 + i)];
  }
}
__device__ __forceinline__ void point_grad(const double* L, double* g) {
  const double* A1 = L;
  const double* A2 = L + 20;
  const double* At = L + 40;
  for (int i = 0; i < 3; ++i) {
    g[i] = A1[6 + i] * L[18] + A1[15 + i] * L[19];
    g[3 + i] = A2[6 + i] * L[38] + A2[15 + i] * L[39];
  }
  if (L[79] != 0.0)
    for (int i = 0; i < 6; ++i) g[i] += At[i] * L[76] + At[12 + i] * L[77] + At[24 + i] * L[78];
}
// undamped pose-pose entry (a >= b) and pose gradient entry of one tracklet
__device__ __forceinline__ double pose_entry(const double* L, int a, int b) {
  const double* A1 = L;
  const double* A2 = L + 20;
  const double* At = L + 40;
  if (a < 6) return A1[a] * A1[b] + A1[9 + a] * A1[9 + b];
  if (a < 12) return b < 6 ? 0.0 : A2[a - 6] * A2[b - 6] + A2[a + 3] * A2[b + 3];
  if (b < 12 || L[79] == 0.0) return 0.0;
  return At[a - 6] * At[b - 6] + At[a + 6] * At[b + 6] + At[a + 18] * At[b + 18];
}
__device__ __forceinline__ double pose_grad(const double* L, int a) {
  const double* A1 = L;
  const double* A2 = L + 20;
  const double* At = L + 40;
  if (a < 6) return A1[a] * L[18] + A1[9 + a] * L[19];
  if (a < 12) return A2[a - 6] * L[38] + A2[a + 3] * L[39];
  if (L[79] == 0.0) return 0.0;
  return At[a - 6] * L[76] + At[a + 6] * L[77] + At[a + 18] * L[78];
}

struct Batch {
  int n;
  const int32_t* track_start;
  const double* X1;
  const double* X2;
  const double* X1i;  // initial values (= X1 / X2 unless overridden)
  const double* X2i;
  const double* H0;
  const double* K;
  const double* kp1;
  const double* kp2;
  const double* m1;
  const double* m2;
  double* lin;      // kLin per tracklet
  double* pts;      // 2 buffers x 6 per tracklet: [m_{k-1} | m_k]
  uint8_t* active;  // the tracklet's ternary factor is in the graph
  const uint8_t* inactive0;  // initial mask (ternary out of the graph at the start)
  uint8_t* outlier;
  double* H_out;
  long long* prof;  // DYNOREFINE_PROFILE builds: 8 phase tick counters per problem
  dynorefine_result* res;
  double isig_proj, isig_motion, hk, isig_prior;
  int outlier_reject;
  dynohip_lm_params lm;
};

struct Shared {
  double X[2][3][12];  // [buffer][X_{k-1}, X_k, H]
  double Z[2][12];     // prior measurements
  double S[18 * 18];   // reduced system (lower), then its Cholesky factor
  double g[18];
  double dx[18];
  double bprior[12];
  double red[kWin * kRedLd];  // cross-lane reduction of S: [entry][quad]
};

__device__ double total_error(const Batch& B, const Shared& sh, const double* Kp, int pb, int pt, int t0, int t1,
                              int lane) {
  Pose X1, X2, H;
  load_pose(sh.X[pb][0], X1);
  load_pose(sh.X[pb][1], X2);
  load_pose(sh.X[pb][2], H);
  double e = 0.0;
  for (int t = t0 + lane; t < t1; t += kWave) {
    const double* p = B.pts + (2 * static_cast<int64_t>(t) + pt) * 6;
    e += projection(X1, p, Kp, B.kp1 + 2 * t, B.isig_proj, B.hk, nullptr, nullptr);
    e += projection(X2, p + 3, Kp, B.kp2 + 2 * t, B.isig_proj, B.hk, nullptr, nullptr);
    if (B.active[t]) e += ternary(p, p + 3, H, B.isig_motion, B.hk, nullptr, nullptr);
  }
  e = wave_sum(e);
  for (int f = 0; f < 2; ++f) {
    Pose X, Z;
    load_pose(sh.X[pb][f], X);
    load_pose(sh.Z[f], Z);
    double r[6];
    prior_residual(X, Z, r);
    double q = 0.0;
    for (int i = 0; i < 6; ++i) q += (r[i] * B.isig_prior) * (r[i] * B.isig_prior);
    e += 0.5 * q;
  }
  return e;
}

#ifndef DYNOREFINE_WAVES_PER_EU
#define DYNOREFINE_WAVES_PER_EU 1
#endif
__global__ __launch_bounds__(kWave, DYNOREFINE_WAVES_PER_EU)
void k_refine(Batch B) {
  __shared__ Shared sh;
  const int prob = blockIdx.x;
  const int lane = threadIdx.x;
  const int t0 = B.track_start[prob], t1 = B.track_start[prob + 1];
  const double* Kp = B.K + 5 * prob;
  const dynohip_lm_params& prm = B.lm;
  if (lane < 12) {
    sh.X[0][0][lane] = B.X1i[12 * prob + lane];
    sh.X[0][1][lane] = B.X2i[12 * prob + lane];
    sh.X[0][2][lane] = B.H0[12 * prob + lane];
    sh.Z[0][lane] = B.X1[12 * prob + lane];
    sh.Z[1][lane] = B.X2[12 * prob + lane];
  }
  for (int t = t0 + lane; t < t1; t += kWave) {
    double* p = B.pts + 2 * static_cast<int64_t>(t) * 6;
    for (int i = 0; i < 3; ++i) {
      p[i] = B.m1[3 * t + i];
      p[3 + i] = B.m2[3 * t + i];
    }
    B.active[t] = B.inactive0[t] ? 0 : 1;
    B.outlier[t] = 0;
  }
  __syncthreads();
  int pb = 0, pt = 0;  // current pose / point buffers
#ifdef DYNOREFINE_PROFILE
  long long pt_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  long long pt_t = clock64();
#define RPROF(k)                  \
  do {                            \
    const long long n_ = clock64(); \
    pt_acc[k] += n_ - pt_t;       \
    pt_t = n_;                    \
  } while (0)
#else
#define RPROF(k) \
  do {           \
  } while (0)
#endif
  double err = total_error(B, sh, Kp, pb, pt, t0, t1, lane);
  RPROF(0);
  const double err0 = err;
  int it_total = 0, inner_total = 0, status = DYNOREFINE_OK, n_outliers = 0;
  const double lambda_f = prm.lambda_factor;

  for (int round = 0; round < 5; ++round) {
    // ---- NonlinearOptimizer::defaultOptimize ----
    double lambda = prm.lambda_initial;
    int iterations = 0;
    if (!(err <= prm.error_tol) && iterations < prm.max_iterations) {
      double newError = err;
      bool converged = false;
      do {
        const double currentError = newError;
        // ---- LevenbergMarquardtOptimizer::iterate: linearise once ----
        Pose X1, X2, H;
        load_pose(sh.X[pb][0], X1);
        load_pose(sh.X[pb][1], X2);
        load_pose(sh.X[pb][2], H);
        double oldLin = 0.0;
        for (int t = t0 + lane; t < t1; t += kWave) {
          double* L = B.lin + static_cast<int64_t>(t) * kLin;
          const double* p = B.pts + (2 * static_cast<int64_t>(t) + pt) * 6;
          projection(X1, p, Kp, B.kp1 + 2 * t, B.isig_proj, B.hk, L, L + 18);
          projection(X2, p + 3, Kp, B.kp2 + 2 * t, B.isig_proj, B.hk, L + 20, L + 38);
          oldLin += 0.5 * (L[18] * L[18] + L[19] * L[19] + L[38] * L[38] + L[39] * L[39]);
          if (B.active[t]) {
            ternary(p, p + 3, H, B.isig_motion, B.hk, L + 40, L + 76);
            L[79] = 1.0;
            oldLin += 0.5 * (L[76] * L[76] + L[77] * L[77] + L[78] * L[78]);
          } else {
            for (int i = 40; i < 80; ++i) L[i] = 0.0;
          }
        }
        oldLin = wave_sum(oldLin);
        if (lane < 2) {
          Pose X, Z;
          load_pose(sh.X[pb][lane], X);
          load_pose(sh.Z[lane], Z);
          double r[6];
          prior_residual(X, Z, r);
          for (int i = 0; i < 6; ++i) sh.bprior[6 * lane + i] = -r[i] * B.isig_prior;
        }
        __syncthreads();
        for (int i = 0; i < 12; ++i) oldLin += 0.5 * sh.bprior[i] * sh.bprior[i];

        RPROF(1);
        // ---- tryLambda until accepted, gave up or stopped ----
        for (;;) {
          // reduced system: sum_i (B_i - W_i^T C_i^-1 W_i), g_pose - W_i^T C_i^-1 g_i,
          // with C_i = L_i L_i^T: entry (a, b) = B_i(a, b) - z_a . z_b where
          // z_c = L_i^-1 W_i(:, c). W_i is block sparse (X_{k-1} columns touch
          // m_{k-1} only, X_k columns m_k only), so z of an X_k column has its
          // top three rows zero. The 171 entries + 18 gradient entries are
          // emitted in three windows of 63 (whole block pairs each, so that
          // only two z blocks are live at a time) and reduced in two stages:
          // quad sums by DPP, stored to LDS (red[entry][quad]), then lane e
          // sums row e in quad order (fixed order: bit-reproducible).
          double acc[3] = {0.0, 0.0, 0.0};
          bool solved = true;
          auto flush = [&](int grp) {
            __syncthreads();
            if (lane < kWin) {
              const double* row = sh.red + lane * kRedLd;
              double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
#pragma unroll
              for (int j = 0; j < kQuads; j += 4) {
                s0 += row[j];
                s1 += row[j + 1];
                s2 += row[j + 2];
                s3 += row[j + 3];
              }
              acc[grp] += (s0 + s1) + (s2 + s3);
            }
            __syncthreads();
          };
          for (int base = t0; base < t1; base += kWave) {
            const int t = base + lane;
            const bool have = t < t1;
            const double* L = B.lin + static_cast<int64_t>(have ? t : t0) * kLin;
            double C[36];
            const bool lok = point_block(L, lambda, C) || !have;
            if (__any(!lok)) {
              solved = false;
              break;
            }
            auto put = [&](int idx, double v) {
              v = quad_sum(have ? v : 0.0);
              if ((lane & 3) == 0) sh.red[idx * kRedLd + (lane >> 2)] = v;
            };
            double zg[6];
            point_grad(L, zg);
            lower_solve(C, zg);
            double Z2[6][6], Z0[6][6];
#pragma unroll
            for (int c = 0; c < 6; ++c) {
              z_column(L, C, 12 + c, Z2[c]);
              z_column(L, C, c, Z0[c]);
            }
            // window 0: (H, H), (H, X_{k-1}), g_H
#pragma unroll
            for (int i = 0; i < 6; ++i)
#pragma unroll
              for (int j = 0; j <= i; ++j) put(i * (i + 1) / 2 + j, pose_entry(L, 12 + i, 12 + j) - dot6(Z2[i], Z2[j]));
#pragma unroll
            for (int i = 0; i < 6; ++i)
#pragma unroll
              for (int j = 0; j < 6; ++j) put(21 + 6 * i + j, -dot6(Z2[i], Z0[j]));
#pragma unroll
            for (int i = 0; i < 6; ++i) put(57 + i, pose_grad(L, 12 + i) - dot6(Z2[i], zg));
            flush(0);
            // window 1: (X_{k-1}, X_{k-1}), g_{X_{k-1}}, (H, X_k)
#pragma unroll
            for (int i = 0; i < 6; ++i)
#pragma unroll
              for (int j = 0; j <= i; ++j) put(i * (i + 1) / 2 + j, pose_entry(L, i, j) - dot6(Z0[i], Z0[j]));
#pragma unroll
            for (int i = 0; i < 6; ++i) put(57 + i, pose_grad(L, i) - dot6(Z0[i], zg));
            double Z1[6][3];
#pragma unroll
            for (int c = 0; c < 6; ++c) z_column_bot(L, C, 6 + c, Z1[c]);
#pragma unroll
            for (int i = 0; i < 6; ++i)
#pragma unroll
              for (int j = 0; j < 6; ++j) put(21 + 6 * i + j, -dot3(Z2[i] + 3, Z1[j]));
            flush(1);
            // window 2: (X_k, X_{k-1}), (X_k, X_k), g_{X_k}; z of the
            // X_{k-1} columns recomputed rather than kept live
            double Z0b[6][6];
#pragma unroll
            for (int c = 0; c < 6; ++c) z_column(L, C, c, Z0b[c]);
#pragma unroll
            for (int i = 0; i < 6; ++i)
#pragma unroll
              for (int j = 0; j < 6; ++j) put(6 * i + j, -dot3(Z1[i], Z0b[j] + 3));
#pragma unroll
            for (int i = 0; i < 6; ++i)
#pragma unroll
              for (int j = 0; j <= i; ++j) put(36 + i * (i + 1) / 2 + j, pose_entry(L, 6 + i, 6 + j) - dot3(Z1[i], Z1[j]));
#pragma unroll
            for (int i = 0; i < 6; ++i) put(57 + i, pose_grad(L, 6 + i) - dot3(Z1[i], zg + 3));
            flush(2);
          }
          if (solved) {
#pragma unroll
            for (int grp = 0; grp < 3; ++grp) {
              if (lane >= kWin) continue;
              int a, b;
              if (lane >= 57) {
                sh.g[(grp == 0 ? 12 : grp == 1 ? 0 : 6) + lane - 57] = acc[grp];
                continue;
              }
              if (grp == 2 && lane < 36) {
                a = 6 + lane / 6;
                b = lane % 6;
              } else if (grp < 2 && lane >= 21) {
                a = 12 + (lane - 21) / 6;
                b = (grp == 0 ? 0 : 6) + (lane - 21) % 6;
              } else {
                const int k = grp == 2 ? lane - 36 : lane;
                const int r = static_cast<int>((sqrt(8.0 * k + 1.0) - 1.0) * 0.5);
                const int off = grp == 0 ? 12 : grp == 1 ? 0 : 6;
                a = off + r;
                b = off + k - r * (r + 1) / 2;
              }
              sh.S[18 * a + b] = acc[grp];
            }
          }
          __syncthreads();
          RPROF(2);
          // priors (J = I / sigma) and damping, then the 18x18 Cholesky in
          // registers: lane i < 18 holds row i; column k is broadcast with
          // readlane. Solves: forward on the rows, backward on the columns
          // (read back from LDS).
          if (solved) {
            const int i = lane < 18 ? lane : 17;
            double r[18];
#pragma unroll
            for (int j = 0; j < 18; ++j) r[j] = j <= i ? sh.S[18 * i + j] : 0.0;
            double gi = sh.g[i];
            const double ip2 = B.isig_prior * B.isig_prior;
#pragma unroll
            for (int j = 0; j < 18; ++j)
              if (j == lane) {
                if (j < 12) {
                  r[j] += ip2;
                  gi += B.isig_prior * sh.bprior[j];
                }
                r[j] += lambda;
              }
            bool fail = false;
#pragma unroll
            for (int k = 0; k < 18; ++k) {
              const double d = read_lane(r[k], k);
              if (!(d > 0.0)) {
                fail = true;
                break;
              }
              const double ld = sqrt(d);
              r[k] = lane == k ? ld : r[k] / ld;
#pragma unroll
              for (int j = k + 1; j < 18; ++j) {
                const double ljk = read_lane(r[k], j);
                if (lane >= j) r[j] -= r[k] * ljk;
              }
            }
            if (fail) {
              solved = false;
            } else {
#pragma unroll
              for (int k = 0; k < 18; ++k) {
                if (lane == k) gi = gi / r[k];
                const double yk = read_lane(gi, k);
                if (lane > k) gi -= r[k] * yk;
              }
              if (lane < 18) {
#pragma unroll
                for (int j = 0; j < 18; ++j)
                  if (j <= lane) sh.S[18 * lane + j] = r[j];
              }
              __syncthreads();
              double ct[18];  // column `lane` of L
#pragma unroll
              for (int m = 0; m < 18; ++m) ct[m] = (m >= i) ? sh.S[18 * m + i] : 0.0;
#pragma unroll
              for (int m = 17; m >= 0; --m) {
                if (lane == m) gi = gi / ct[m];
                const double xm = read_lane(gi, m);
                if (lane < m) gi -= ct[m] * xm;
              }
              if (lane < 18) sh.dx[lane] = gi;
            }
          }
          __syncthreads();
          RPROF(3);
          // back-substitution, linearised error at delta, candidate points
          double newLin = 0.0;
          if (solved) {
            double dx[18];
            for (int i = 0; i < 18; ++i) dx[i] = sh.dx[i];
            for (int t = t0 + lane; t < t1; t += kWave) {
              const double* L = B.lin + static_cast<int64_t>(t) * kLin;
              double C[36];
              point_block(L, lambda, C);
              double r[6];
              point_grad(L, r);
              for (int a = 0; a < 18; ++a) {
                double w[6];
                w_column(L, a, w);
                for (int i = 0; i < 6; ++i) r[i] -= w[i] * dx[a];
              }
              point_solve(C, r);  // r = delta of [m_{k-1} | m_k]
              double e = 0.0;
              for (int row = 0; row < 2; ++row) {
                double s1 = -L[18 + row], s2 = -L[38 + row];
                for (int j = 0; j < 6; ++j) {
                  s1 += L[9 * row + j] * dx[j];
                  s2 += L[20 + 9 * row + j] * dx[6 + j];
                }
                for (int j = 0; j < 3; ++j) {
                  s1 += L[9 * row + 6 + j] * r[j];
                  s2 += L[20 + 9 * row + 6 + j] * r[3 + j];
                }
                e += s1 * s1 + s2 * s2;
              }
              if (L[79] != 0.0)
                for (int row = 0; row < 3; ++row) {
                  const double* A = L + 40 + 12 * row;
                  double s = -L[76 + row];
                  for (int j = 0; j < 6; ++j) s += A[j] * r[j];
                  for (int j = 0; j < 6; ++j) s += A[6 + j] * dx[12 + j];
                  e += s * s;
                }
              newLin += 0.5 * e;
              const double* p = B.pts + (2 * static_cast<int64_t>(t) + pt) * 6;
              double* pc = B.pts + (2 * static_cast<int64_t>(t) + (1 - pt)) * 6;
              for (int i = 0; i < 6; ++i) pc[i] = p[i] + r[i];
            }
            newLin = wave_sum(newLin);
            for (int i = 0; i < 12; ++i) {
              const double s = B.isig_prior * dx[i] - sh.bprior[i];
              newLin += 0.5 * s * s;
            }
          }
          bool step_ok = false, stop = false;
          double newErr = INFINITY;
          if (solved && isfinite(newLin)) {
            const double linChange = oldLin - newLin;
            if (linChange >= 0) {
              if (lane < 3) {
                Pose T, Tn;
                load_pose(sh.X[pb][lane], T);
                pose_retract(T, sh.dx + 6 * lane, Tn);
                store_pose(sh.X[1 - pb][lane], Tn);
              }
              __syncthreads();
              RPROF(4);
              newErr = total_error(B, sh, Kp, 1 - pb, 1 - pt, t0, t1, lane);
              RPROF(5);
              const double costChange = err - newErr;
              if (linChange > DBL_EPSILON * oldLin) step_ok = costChange / linChange > prm.min_model_fidelity;
              if (fabs(costChange) < prm.relative_error_tol * err) stop = true;
            }
          }
          __syncthreads();
          if (step_ok) {
            ++inner_total;
            pb = 1 - pb;
            pt = 1 - pt;
            err = newErr;
            lambda /= lambda_f;
            if (lambda < prm.lambda_lower_bound) lambda = prm.lambda_lower_bound;
            ++iterations;
            break;
          } else if (!stop) {
            ++inner_total;
            lambda *= lambda_f;
            if (lambda >= prm.lambda_upper_bound) break;
          } else {
            break;
          }
        }
        newError = err;
        // NonlinearOptimizer::checkConvergence
        if (newError <= prm.error_tol) {
          converged = true;
        } else {
          const double absd = currentError - newError;
          converged = (absd / currentError <= prm.relative_error_tol) || (absd <= prm.absolute_error_tol);
        }
        if (!(iterations < prm.max_iterations && !converged && isfinite(currentError))) break;
      } while (true);
    }
    it_total += iterations;
    // ---- determineFactorOutliers<LandmarkMotionTernaryFactor> ----
    if (B.outlier_reject == 0) break;
    Pose H;
    load_pose(sh.X[pb][2], H);
    int cnt = 0;
    for (int t = t0 + lane; t < t1; t += kWave) {
      if (!B.active[t]) continue;
      const double* p = B.pts + (2 * static_cast<int64_t>(t) + pt) * 6;
      double ge;
      ternary(p, p + 3, H, B.isig_motion, B.hk, nullptr, nullptr, &ge);
      if (ge > 0.5 * kChi2_3_099) ++cnt;
    }
    cnt = static_cast<int>(wave_sum(static_cast<double>(cnt)));
    if (cnt == 0) break;
    if (B.outlier_reject == 1 || round == 4) {
      if (B.outlier_reject == 1) {
        // values.insert(object_motion_key, ...) throws ValuesKeyAlreadyExists
        status = DYNOREFINE_VALUES_KEY_EXISTS;
        for (int t = t0 + lane; t < t1; t += kWave) {
          const double* p = B.pts + (2 * static_cast<int64_t>(t) + pt) * 6;
          double ge;
          ternary(p, p + 3, H, B.isig_motion, B.hk, nullptr, nullptr, &ge);
          if (ge > 0.5 * kChi2_3_099) B.outlier[t] = 1;
        }
        n_outliers = cnt;
      }
      break;
    }
    // outlier_reject == 2: drop the outlier ternary factors and re-solve from
    // the optimised values
    for (int t = t0 + lane; t < t1; t += kWave) {
      if (!B.active[t]) continue;
      const double* p = B.pts + (2 * static_cast<int64_t>(t) + pt) * 6;
      double ge;
      ternary(p, p + 3, H, B.isig_motion, B.hk, nullptr, nullptr, &ge);
      if (ge > 0.5 * kChi2_3_099) {
        B.active[t] = 0;
        B.outlier[t] = 1;
      }
    }
    n_outliers += cnt;
    __syncthreads();
    err = total_error(B, sh, Kp, pb, pt, t0, t1, lane);
  }
  RPROF(6);
#ifdef DYNOREFINE_PROFILE
  if (lane < 8) {
    long long v = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) v = lane == k ? pt_acc[k] : v;
    B.prof[8 * prob + lane] = v;
  }
#endif
  if (lane < 12) B.H_out[12 * prob + lane] = sh.X[pb][2][lane];
  if (lane == 0) {
    dynorefine_result r;
    r.iterations = it_total;
    r.inner_iterations = inner_total;
    r.status = status;
    r.n_outliers = n_outliers;
    r.error_before = err0;
    r.error_after = err;
    B.res[prob] = r;
  }
}

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  hipError_t alloc(size_t count) {
    if (count <= n && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    hipError_t e = hipMalloc(&p, (count ? count : 1) * sizeof(T));
    if (e == hipSuccess) n = count;
    return e;
  }
  hipError_t upload(const T* src, size_t count, hipStream_t s) {
    hipError_t e = alloc(count);
    if (e != hipSuccess || count == 0) return e;
    return hipMemcpyAsync(p, src, count * sizeof(T), hipMemcpyHostToDevice, s);
  }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

}  // namespace

struct dynorefine_solver {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  std::string err;
  size_t n_prob = 0;
  int64_t n_track = 0;
  DevBuf<int32_t> ts;
  DevBuf<double> X1, X2, X1i, X2i, H0, K, kp1, kp2, m1, m2, lin, pts, Hout;
  DevBuf<uint8_t> active, outlier, inactive0;
  DevBuf<dynorefine_result> res;
  float last_ms = 0.f;
  bool solved = false;
};

#define RCHK(s, expr)                                                            \
  do {                                                                           \
    hipError_t e_ = (expr);                                                      \
    if (e_ != hipSuccess) {                                                      \
      (s)->err = std::string(#expr) + ": " + hipGetErrorString(e_);             \
      return DYNOHIP_EHIP;                                                       \
    }                                                                            \
  } while (0)

extern "C" {

void dynorefine_params_default(dynorefine_params* p) {
  if (!p) return;
  p->landmark_motion_sigma = 0.001;
  p->projection_sigma = 2.0;
  p->k_huber = 0.0001;
  p->prior_sigma = 1e-5;
  p->outlier_reject = 1;
  p->reserved = 0;
}

int dynorefine_create(int device_id, dynorefine_solver** out) {
  if (!out) return DYNOHIP_EINVAL;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device_id < 0 || device_id >= n) return DYNOHIP_EHIP;
  auto* s = new dynorefine_solver();
  s->device = device_id;
  if (hipSetDevice(device_id) != hipSuccess || hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&s->ev[0]) != hipSuccess || hipEventCreate(&s->ev[1]) != hipSuccess) {
    delete s;
    return DYNOHIP_EHIP;
  }
  *out = s;
  return DYNOHIP_OK;
}

void dynorefine_destroy(dynorefine_solver* s) {
  if (!s) return;
  (void)hipSetDevice(s->device);
  if (s->stream) (void)hipStreamSynchronize(s->stream);
  for (auto& e : s->ev)
    if (e) (void)hipEventDestroy(e);
  if (s->stream) (void)hipStreamDestroy(s->stream);
  delete s;
}

const char* dynorefine_last_error(const dynorefine_solver* s) { return s ? s->err.c_str() : "null solver"; }

int dynorefine_upload(dynorefine_solver* s, const dynorefine_batch* b) {
  if (!s || !b || !b->track_start || (b->n_problems && (!b->X_k_1 || !b->X_k || !b->H_init || !b->calibration))) {
    if (s) s->err = "invalid batch";
    return DYNOHIP_EINVAL;
  }
  RCHK(s, hipSetDevice(s->device));
  const size_t n = b->n_problems;
  if (b->track_start[0] != 0) {
    s->err = "track_start[0] must be 0";
    return DYNOHIP_EINVAL;
  }
  for (size_t p = 0; p < n; ++p)
    if (b->track_start[p + 1] < b->track_start[p]) {
      s->err = "track_start is not ascending";
      return DYNOHIP_EINVAL;
    }
  const int64_t nt = b->track_start[n];
  if (nt > 0 && (!b->kp_k_1 || !b->kp_k || !b->m_k_1 || !b->m_k)) {
    s->err = "null tracklet arrays";
    return DYNOHIP_EINVAL;
  }
  for (size_t i = 0; i < 12 * n; ++i)
    if (!std::isfinite(b->X_k_1[i]) || !std::isfinite(b->X_k[i]) || !std::isfinite(b->H_init[i])) {
      s->err = "non-finite pose";
      return DYNOHIP_ENONFINITE;
    }
  for (int64_t i = 0; i < 3 * nt; ++i)
    if (!std::isfinite(b->m_k_1[i]) || !std::isfinite(b->m_k[i])) {
      s->err = "non-finite point";
      return DYNOHIP_ENONFINITE;
    }
  hipStream_t st = s->stream;
  RCHK(s, s->ts.upload(b->track_start, n + 1, st));
  RCHK(s, s->X1.upload(b->X_k_1, 12 * n, st));
  RCHK(s, s->X2.upload(b->X_k, 12 * n, st));
  RCHK(s, s->X1i.upload(b->X_k_1_init ? b->X_k_1_init : b->X_k_1, 12 * n, st));
  RCHK(s, s->X2i.upload(b->X_k_init ? b->X_k_init : b->X_k, 12 * n, st));
  RCHK(s, s->H0.upload(b->H_init, 12 * n, st));
  RCHK(s, s->K.upload(b->calibration, 5 * n, st));
  RCHK(s, s->kp1.upload(b->kp_k_1, 2 * nt, st));
  RCHK(s, s->kp2.upload(b->kp_k, 2 * nt, st));
  RCHK(s, s->m1.upload(b->m_k_1, 3 * nt, st));
  RCHK(s, s->m2.upload(b->m_k, 3 * nt, st));
  RCHK(s, s->lin.alloc(static_cast<size_t>(kLin) * (nt ? nt : 1)));
  RCHK(s, s->pts.alloc(12 * static_cast<size_t>(nt ? nt : 1)));
  RCHK(s, s->active.alloc(nt ? nt : 1));
  RCHK(s, s->inactive0.alloc(nt ? nt : 1));
  if (b->ternary_inactive && nt)
    RCHK(s, hipMemcpyAsync(s->inactive0.p, b->ternary_inactive, nt, hipMemcpyHostToDevice, st));
  else
    RCHK(s, hipMemsetAsync(s->inactive0.p, 0, nt ? nt : 1, st));
  RCHK(s, s->outlier.alloc(nt ? nt : 1));
  RCHK(s, s->Hout.alloc(12 * (n ? n : 1)));
  RCHK(s, s->res.alloc(n ? n : 1));
  RCHK(s, hipStreamSynchronize(st));
  s->n_prob = n;
  s->n_track = nt;
  s->solved = false;
  return DYNOHIP_OK;
}

int dynorefine_solve(dynorefine_solver* s, const dynorefine_params* p, const dynohip_lm_params* lm) {
  if (!s) return DYNOHIP_EINVAL;
  dynorefine_params prm;
  dynorefine_params_default(&prm);
  if (p) prm = *p;
  dynohip_lm_params lmp;
  dynohip_lm_params_default(&lmp);
  if (lm) lmp = *lm;
  if (!(prm.landmark_motion_sigma > 0 && prm.projection_sigma > 0 && prm.prior_sigma > 0 && prm.k_huber > 0) ||
      prm.outlier_reject < 0 || prm.outlier_reject > 2) {
    s->err = "invalid refinement parameters";
    return DYNOHIP_EINVAL;
  }
  RCHK(s, hipSetDevice(s->device));
  Batch B;
  B.n = static_cast<int>(s->n_prob);
  B.track_start = s->ts.p;
  B.X1 = s->X1.p;
  B.X2 = s->X2.p;
  B.X1i = s->X1i.p;
  B.X2i = s->X2i.p;
  B.H0 = s->H0.p;
  B.K = s->K.p;
  B.kp1 = s->kp1.p;
  B.kp2 = s->kp2.p;
  B.m1 = s->m1.p;
  B.m2 = s->m2.p;
  B.lin = s->lin.p;
  B.pts = s->pts.p;
  B.active = s->active.p;
  B.inactive0 = s->inactive0.p;
  B.outlier = s->outlier.p;
  B.H_out = s->Hout.p;
  B.res = s->res.p;
  B.prof = nullptr;
#ifdef DYNOREFINE_PROFILE
  DevBuf<long long> prof;
  RCHK(s, prof.alloc(8 * s->n_prob));
  B.prof = prof.p;
#endif
  B.isig_proj = 1.0 / prm.projection_sigma;
  B.isig_motion = 1.0 / prm.landmark_motion_sigma;
  B.hk = prm.k_huber;
  B.isig_prior = 1.0 / prm.prior_sigma;
  B.outlier_reject = prm.outlier_reject;
  B.lm = lmp;
  RCHK(s, hipEventRecord(s->ev[0], s->stream));
  if (s->n_prob > 0) k_refine<<<dim3(static_cast<unsigned>(s->n_prob)), dim3(kWave), 0, s->stream>>>(B);
  RCHK(s, hipGetLastError());
  RCHK(s, hipEventRecord(s->ev[1], s->stream));
  RCHK(s, hipEventSynchronize(s->ev[1]));
  RCHK(s, hipEventElapsedTime(&s->last_ms, s->ev[0], s->ev[1]));
#ifdef DYNOREFINE_PROFILE
  {
    std::vector<long long> h(8 * s->n_prob);
    RCHK(s, hipMemcpy(h.data(), prof.p, h.size() * sizeof(long long), hipMemcpyDeviceToHost));
    double tot[8] = {0};
    for (size_t p = 0; p < s->n_prob; ++p)
      for (int k = 0; k < 8; ++k) tot[k] += static_cast<double>(h[8 * p + k]);
    std::fprintf(stderr, "[refine profile] mean clock64 ticks per problem:");
    const char* names[8] = {"init_error", "linearize", "schur", "solve18", "backsub", "new_error", "rest", "-"};
    for (int k = 0; k < 7; ++k) std::fprintf(stderr, " %s=%.0f", names[k], tot[k] / std::max<size_t>(1, s->n_prob));
    std::fprintf(stderr, "\n");
  }
#endif
  s->solved = true;
  return DYNOHIP_OK;
}

int dynorefine_download(dynorefine_solver* s, double* H_out, uint8_t* outlier_out, dynorefine_result* results) {
  if (!s) return DYNOHIP_EINVAL;
  if (!s->solved) {
    s->err = "no solve to download";
    return DYNOHIP_ESTATE;
  }
  RCHK(s, hipSetDevice(s->device));
  if (H_out && s->n_prob)
    RCHK(s, hipMemcpyAsync(H_out, s->Hout.p, 12 * s->n_prob * sizeof(double), hipMemcpyDeviceToHost, s->stream));
  if (outlier_out && s->n_track)
    RCHK(s, hipMemcpyAsync(outlier_out, s->outlier.p, s->n_track, hipMemcpyDeviceToHost, s->stream));
  if (results && s->n_prob)
    RCHK(s, hipMemcpyAsync(results, s->res.p, s->n_prob * sizeof(dynorefine_result), hipMemcpyDeviceToHost,
                           s->stream));
  RCHK(s, hipStreamSynchronize(s->stream));
  return DYNOHIP_OK;
}

int dynorefine_run(dynorefine_solver* s, const dynorefine_batch* b, const dynorefine_params* p,
                   const dynohip_lm_params* lm, double* H_out, uint8_t* outlier_out, dynorefine_result* results) {
  int rc = dynorefine_upload(s, b);
  if (rc == DYNOHIP_OK) rc = dynorefine_solve(s, p, lm);
  if (rc == DYNOHIP_OK) rc = dynorefine_download(s, H_out, outlier_out, results);
  return rc;
}

double dynorefine_last_solve_ms(const dynorefine_solver* s) { return s ? s->last_ms : 0.0; }

}  // extern "C"
