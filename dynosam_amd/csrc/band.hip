// band.hip — block-banded Cholesky of the reduced (Schur) pose system and
// its triangular solves: 64x64 FP64 tiles, lower band stored by column tile
// (tile (j+d, j) at off[j] + d*4096, row-major), D_j sub-diagonal tiles.
//
// One launch per column tile j, k_step(j), with two kinds of workgroups:
//   panel blocks d = 0..D_j   apply column j-1's contribution to their own
//       tile (j+d, j) and to the diagonal tile (j, j) (right-looking update,
//       so no other launch is needed for column j), factor the diagonal
//       tile in registers (4x4-blocked: one thread factors and inverts each
//       4x4 diagonal sub-block, two barriers per 4 pivots) together with
//       L_jj^-1, and then
//         d == 0: store L_jj^-1 and y_j = L_jj^-1 r_j (forward substitution
//                 fused into the factorisation),
//         d >= 1: L(j+d, j) = A L_jj^-T (FP64 MFMA GEMM with the explicit
//                 inverse), r_{j+d} -= L(j+d, j) y_j;
//   update blocks             the rest of column j-1's trailing update:
//       tile (j-1+d1, j-1+d2) -= L(j-1+d1, j-1) L(j-1+d2, j-1)^T, d2 >= 2.
// Every tile receives each column's contribution exactly once and no
// workgroup writes what another workgroup of the same launch reads, so the
// result is deterministic. k_band_back then runs
// x_j = L_jj^-T (y_j - sum_d L(j+d,j)^T x_{j+d}) in one workgroup.
// A non-positive pivot sets *fail (the LM treats the step as failed:
// GTSAM's IndeterminantLinearSystemException path).
#include <hip/hip_runtime.h>

#include "kernels.hpp"

namespace dynohip {

namespace {

constexpr int T = kTile;
constexpr int LD = T + 4;            // padded LDS row stride (doubles)

typedef double v4d __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void load_tile_lds(const double* __restrict__ src, double* dst, int tid, int nthreads) {
  const double2* s2 = reinterpret_cast<const double2*>(src);
  for (int e = tid; e < T * T / 2; e += nthreads) {
    const double2 v = s2[e];
    const int r = (2 * e) / T, c = (2 * e) % T;
    dst[r * LD + c] = v.x;
    dst[r * LD + c + 1] = v.y;
  }
}

// 64x64x64 C = A B^T on LDS operands with v_mfma_f64_16x16x4f64; waves 0..3
// each own a 32x32 quadrant (2x2 MFMA tiles). Lane l feeds A[i0+(l&15)][k0+(l>>4)]
// and B[j0+(l&15)][k0+(l>>4)]; result acc[ti][tj][r] = C[i0+16ti+(l>>4)+4r][j0+16tj+(l&15)].
__device__ __forceinline__ void mfma_abt(const double* As, const double* Bs, int wave, int lane, v4d acc[2][2]) {
  const int i0 = 32 * (wave >> 1), j0 = 32 * (wave & 1);
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
  for (int k0 = 0; k0 < T; k0 += 4) {
    const int k = k0 + lk;
    const double a0 = As[(i0 + li) * LD + k], a1 = As[(i0 + 16 + li) * LD + k];
    const double b0 = Bs[(j0 + li) * LD + k], b1 = Bs[(j0 + 16 + li) * LD + k];
    acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
  }
}

// element (row, col) of the quadrant result held by this lane
#define MFMA_ROW(wave, lane, ti, r) (32 * ((wave) >> 1) + 16 * (ti) + ((lane) >> 4) + 4 * (r))
#define MFMA_COL(wave, lane, tj) (32 * ((wave) & 1) + 16 * (tj) + ((lane) & 15))

__device__ __forceinline__ double pivot_ok(double x, bool& ok) {
  if (!(x > 0.0) || !isfinite(x)) {
    ok = false;
    return 1.0;
  }
  return x;
}

// 1/sqrt(x): hardware estimate + two Newton steps (full FP64 accuracy)
__device__ __forceinline__ double rsqrt_nr(double x) {
  double y = __builtin_amdgcn_rsq(x);
  y = y * (1.5 - 0.5 * x * y * y);
  y = y * (1.5 - 0.5 * x * y * y);
  return y;
}

// 4x4 Cholesky + inverse of a lower 4x4 (row-major a[4][4]); m receives
// L^-1 (lower). Only the reciprocal pivots r_i = 1/l_ii are formed.
// ok is cleared on a non-positive pivot.
__device__ __forceinline__ void chol_inv4(const double (&a)[4][4], double (&m)[4][4], bool& ok) {
  const double r0 = rsqrt_nr(pivot_ok(a[0][0], ok));
  const double l10 = a[1][0] * r0, l20 = a[2][0] * r0, l30 = a[3][0] * r0;
  const double r1 = rsqrt_nr(pivot_ok(a[1][1] - l10 * l10, ok));
  const double l21 = (a[2][1] - l20 * l10) * r1, l31 = (a[3][1] - l30 * l10) * r1;
  const double r2 = rsqrt_nr(pivot_ok(a[2][2] - l20 * l20 - l21 * l21, ok));
  const double l32 = (a[3][2] - l30 * l20 - l31 * l21) * r2;
  const double r3 = rsqrt_nr(pivot_ok(a[3][3] - l30 * l30 - l31 * l31 - l32 * l32, ok));
  m[0][0] = r0; m[1][1] = r1; m[2][2] = r2; m[3][3] = r3;
  m[1][0] = -r1 * (l10 * r0);
  m[2][1] = -r2 * (l21 * r1);
  m[3][2] = -r3 * (l32 * r2);
  m[2][0] = -r2 * (l20 * r0 + l21 * m[1][0]);
  m[3][1] = -r3 * (l31 * r1 + l32 * m[2][1]);
  m[3][0] = -r3 * (l30 * r0 + l31 * m[1][0] + l32 * m[2][0]);
  m[0][1] = m[0][2] = m[0][3] = m[1][2] = m[1][3] = m[2][3] = 0.0;
}

__device__ __forceinline__ double* tile_ptr(const BandDev& b, int i, int j) {
  return b.band + b.off[j] + static_cast<int64_t>(i - j) * T * T;
}

// MFMA accumulator layout of a 64x64 tile over 4 waves: wave w holds the 16
// rows 16w.. as four 16x16 tiles TJ; lane l, reg r of tile TJ is element
// (16w + (l>>4) + 4r, 16TJ + (l&15)).
#define ACC_ROW(w, l, r) (16 * (w) + ((l) >> 4) + 4 * (r))
#define ACC_COL(TJ, l) (16 * (TJ) + ((l) & 15))

// Factor the diagonal tile held in accumulator layout (accA) and build its
// inverse (accX, starting from I). Right-looking, 4 pivots per step:
//   publish column block kb of A and row block kb of the running inverse
//   to LDS (double-buffered), one barrier; every lane forms M = L_kk^-1
//   (4x4) redundantly, the panel entries it feeds to the MFMAs
//   (L = A_panel M^T, zero for rows <= 4kb+3) and the finalised inverse
//   rows Xf = M X_kb; then accA -= L L^T and accX -= L Xf (4+4
//   v_mfma_f64_16x16x4 per wave) and X rows 4kb.. are replaced by Xf.
__device__ bool factor_tile_mfma(v4d (&accA)[4], v4d (&accX)[4], int w, int l, double* Pcol, double* Xrow) {
  bool ok = true;
  const int li = l & 15, lk = l >> 4;
  for (int KB = 0; KB < 4; ++KB) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int kb = 4 * KB + kk, p = kk & 1;
      double* P = Pcol + p * (T * 4);
      double* X = Xrow + p * (4 * T);
      // publish A[:, 4kb..4kb+3] (tile column KB, in-tile cols 4kk..4kk+3)
      if (li >= 4 * kk && li < 4 * kk + 4) {
#pragma unroll
        for (int r = 0; r < 4; ++r) P[ACC_ROW(w, l, r) * 4 + (li - 4 * kk)] = accA[KB][r];
      }
      // publish X[4kb..4kb+3, :] (wave KB, register kk)
      if (w == KB) {
#pragma unroll
        for (int TJ = 0; TJ < 4; ++TJ) X[lk * T + ACC_COL(TJ, l)] = accX[TJ][kk];
      }
      __syncthreads();
      // M = L_kk^-1 of the 4x4 pivot block (every lane, redundantly)
      double a4[4][4], M[4][4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int q = 0; q < 4; ++q) a4[u][q] = P[(4 * kb + u) * 4 + q];
      chol_inv4(a4, M, ok);
      // panel entries fed to the MFMAs: L[i][k] = sum_{m<=k} A[i][m] M[k][m]
      auto panel = [&](int i) {
        double s = 0.0;
#pragma unroll
        for (int m = 0; m < 4; ++m) s += P[i * 4 + m] * M[lk][m];
        return i > 4 * kb + 3 ? s : 0.0;
      };
      const double aL = -panel(16 * w + li);
      double bL[4], xf[4];
#pragma unroll
      for (int TJ = 0; TJ < 4; ++TJ) {
        bL[TJ] = panel(16 * TJ + li);
        double s = 0.0;
#pragma unroll
        for (int m = 0; m < 4; ++m) s += M[lk][m] * X[m * T + ACC_COL(TJ, l)];
        xf[TJ] = s;
      }
      // only active 16x16 tiles: rows > 4kb+3 (w >= KB); A lower (KB <= TJ <= w),
      // inverse columns <= 4kb+3 (TJ <= KB)
      if (w >= KB) {
#pragma unroll
        for (int TJ = 0; TJ < 4; ++TJ) {
          if (TJ >= KB && TJ <= w) accA[TJ] = __builtin_amdgcn_mfma_f64_16x16x4f64(aL, bL[TJ], accA[TJ], 0, 0, 0);
          if (TJ <= KB) accX[TJ] = __builtin_amdgcn_mfma_f64_16x16x4f64(aL, xf[TJ], accX[TJ], 0, 0, 0);
        }
      }
      if (w == KB) {
#pragma unroll
        for (int TJ = 0; TJ < 4; ++TJ) accX[TJ][kk] = xf[TJ];
      }
    }
  }
  return ok;
}

// y = L^-1 v (64, L^-1 in LDS with stride LD, lower): 4 lanes per row
__device__ __forceinline__ double lower_gemv4(const double* Li, const double* v, int tid) {
  const int row = tid >> 2, part = tid & 3;
  double s = 0.0;
  for (int m = part; m <= row; m += 4) s += Li[row * LD + m] * v[m];
  s += __shfl_xor(s, 1);
  s += __shfl_xor(s, 2);
  return s;
}

__global__ __launch_bounds__(256) void k_step(BandDev b, int j, int npanel, double* __restrict__ Linv,
                                              double* __restrict__ r, double* __restrict__ y, int* fail) {
  __shared__ double Ps[T * LD];   // L(j, j-1)  -> later L_jj^-1
  __shared__ double Qs[T * LD];   // L(j+d, j-1) / update operand
  __shared__ double As[T * LD];   // tile (j+d, j)
  __shared__ double Pcol[2 * T * 4];
  __shared__ double Xrow[2 * 4 * T];
  __shared__ double vv[T];
  const int tid = threadIdx.x;
  const int w = tid >> 6, l = tid & 63;
  const int Dprev = j > 0 ? b.D[j - 1] : 0;
  if (static_cast<int>(blockIdx.x) >= npanel) {
    // ---- update block: tile (j-1+d1, j-1+d2) -= L(j-1+d1, j-1) L(j-1+d2, j-1)^T, d2 >= 2
    int t = blockIdx.x - npanel, d1 = 2;
    while (t >= d1 - 1) { t -= d1 - 1; ++d1; }
    const int d2 = t + 2;
    load_tile_lds(tile_ptr(b, j - 1 + d1, j - 1), Qs, tid, 256);
    load_tile_lds(tile_ptr(b, j - 1 + d2, j - 1), Ps, tid, 256);
    __syncthreads();
    v4d acc[2][2];
    mfma_abt(Qs, Ps, w, l, acc);
    double* dst = tile_ptr(b, j - 1 + d1, j - 1 + d2);
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < 2; ++tj)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) dst[MFMA_ROW(w, l, ti, rr) * T + MFMA_COL(w, l, tj)] -= acc[ti][tj][rr];
    return;
  }
  // ---- panel block d
  const int d = blockIdx.x;
  const bool has_prev = Dprev >= 1;             // tile (j, j-1) exists
  const bool prev_d = d > 0 && Dprev >= d + 1;  // tile (j+d, j-1) exists
  if (has_prev) load_tile_lds(tile_ptr(b, j, j - 1), Ps, tid, 256);
  if (d > 0) load_tile_lds(tile_ptr(b, j + d, j), As, tid, 256);
  if (prev_d) load_tile_lds(tile_ptr(b, j + d, j - 1), Qs, tid, 256);
  v4d accA[4], accX[4];
  const double* diag = tile_ptr(b, j, j);
#pragma unroll
  for (int TJ = 0; TJ < 4; ++TJ)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = ACC_ROW(w, l, rr), col = ACC_COL(TJ, l);
      accA[TJ][rr] = diag[row * T + col];
      accX[TJ][rr] = row == col ? 1.0 : 0.0;
    }
  __syncthreads();
  const int li = l & 15, lk = l >> 4;
  if (has_prev) {
    // A_jj -= L(j,j-1) L(j,j-1)^T into the accumulators (K = 64)
#pragma unroll 4
    for (int k0 = 0; k0 < T; k0 += 4) {
      const double a = -Ps[(16 * w + li) * LD + k0 + lk];
#pragma unroll
      for (int TJ = 0; TJ < 4; ++TJ)
        accA[TJ] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Ps[(16 * TJ + li) * LD + k0 + lk], accA[TJ], 0, 0, 0);
    }
  }
  if (prev_d) {
    // A_dj -= L(j+d,j-1) L(j,j-1)^T
    v4d acc[2][2];
    mfma_abt(Qs, Ps, w, l, acc);
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < 2; ++tj)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) As[MFMA_ROW(w, l, ti, rr) * LD + MFMA_COL(w, l, tj)] -= acc[ti][tj][rr];
  }
  __syncthreads();
  const bool ok = factor_tile_mfma(accA, accX, w, l, Pcol, Xrow);
  if (!ok && d == 0 && tid == 0) *fail = 1;
  // L_jj^-1 -> Ps (full square; upper part is exactly zero)
#pragma unroll
  for (int TJ = 0; TJ < 4; ++TJ)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) Ps[ACC_ROW(w, l, rr) * LD + ACC_COL(TJ, l)] = accX[TJ][rr];
  if (d == 0) {
    double* dst = Linv + static_cast<int64_t>(j) * T * T;
#pragma unroll
    for (int TJ = 0; TJ < 4; ++TJ)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) dst[ACC_ROW(w, l, rr) * T + ACC_COL(TJ, l)] = accX[TJ][rr];
  }
  const double* rj = r + static_cast<int64_t>(j) * T;
  if (tid < T) vv[tid] = rj[tid];
  __syncthreads();
  // y_j = L_jj^-1 r_j
  const double yrow = lower_gemv4(Ps, vv, tid);
  __syncthreads();
  if ((tid & 3) == 0) {
    vv[tid >> 2] = yrow;
    if (d == 0) y[static_cast<int64_t>(j) * T + (tid >> 2)] = yrow;
  }
  if (d == 0) return;
  // L(j+d, j) = A L^-T
  v4d acc[2][2];
  mfma_abt(As, Ps, w, l, acc);
  __syncthreads();
  double* dst = tile_ptr(b, j + d, j);
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < 2; ++tj)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = MFMA_ROW(w, l, ti, rr), col = MFMA_COL(w, l, tj);
        dst[row * T + col] = acc[ti][tj][rr];
        As[row * LD + col] = acc[ti][tj][rr];
      }
  __syncthreads();
  // r_{j+d} -= L(j+d, j) y_j (4 lanes per row)
  {
    const int row = tid >> 2, part = tid & 3;
    double s = 0.0;
    for (int m = part; m < T; m += 4) s += As[row * LD + m] * vv[m];
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    if (part == 0) r[static_cast<int64_t>(j + d) * T + row] -= s;
  }
}

// backward substitution with the stored inverses (one workgroup)
constexpr int kBackThreads = 1024;
__global__ __launch_bounds__(kBackThreads) void k_band_back(BandDev b, const double* __restrict__ Linv,
                                                            const double* __restrict__ y, double* __restrict__ x) {
  constexpr int NP = kBackThreads / T;  // 16 parts
  __shared__ double part[NP][T];
  __shared__ double rv[T];
  const int tid = threadIdx.x, c = tid & (T - 1), q = tid >> 6;
  for (int i = b.NT - 1; i >= 0; --i) {
    const int D = b.D[i];
    // sum_d sum_m L(i+d, i)[m][c] x_{i+d}[m]; the D*64 (d, m) rows are split
    // over 16 parts, 4 independent loads in flight per thread
    const double* col = b.band + b.off[i] + static_cast<int64_t>(T) * T;
    const double* xs = x + static_cast<int64_t>(i + 1) * T;
    const int nrow = D * T;
    double s = 0.0, s1 = 0.0, s2a = 0.0, s3 = 0.0;
    int row = q;
    for (; row + 3 * NP < nrow; row += 4 * NP) {
      const double a0 = col[static_cast<int64_t>(row) * T + c], a1 = col[static_cast<int64_t>(row + NP) * T + c];
      const double a2 = col[static_cast<int64_t>(row + 2 * NP) * T + c], a3 = col[static_cast<int64_t>(row + 3 * NP) * T + c];
      s += a0 * xs[row];
      s1 += a1 * xs[row + NP];
      s2a += a2 * xs[row + 2 * NP];
      s3 += a3 * xs[row + 3 * NP];
    }
    for (; row < nrow; row += NP) s += col[static_cast<int64_t>(row) * T + c] * xs[row];
    s = (s + s1) + (s2a + s3);
    part[q][c] = s;
    __syncthreads();
    if (tid < T) {
      double t2 = 0.0;
#pragma unroll
      for (int k = 0; k < NP; ++k) t2 += part[k][tid];
      rv[tid] = y[static_cast<int64_t>(i) * T + tid] - t2;
    }
    __syncthreads();
    // x_i = Linv^T rv : x[c] = sum_{m >= c} Linv[m][c] rv[m]
    const double* Li = Linv + static_cast<int64_t>(i) * T * T;
    double s2 = 0.0;
    for (int m = q; m < T; m += NP)
      if (m >= c) s2 += Li[m * T + c] * rv[m];
    part[q][c] = s2;
    __syncthreads();
    if (tid < T) {
      double t3 = 0.0;
#pragma unroll
      for (int k = 0; k < NP; ++k) t3 += part[k][tid];
      x[static_cast<int64_t>(i) * T + tid] = t3;
    }
    __syncthreads();
  }
}

}  // namespace

void launch_band_cholesky_solve(const BandDev& b, const int32_t* host_D, double* Linv, double* r, double* y,
                                double* x, int* fail, hipStream_t s) {
  for (int j = 0; j < b.NT; ++j) {
    const int npanel = host_D[j] + 1;
    const int Dp = j > 0 ? host_D[j - 1] : 0;
    const int nupd = Dp >= 2 ? (Dp - 1) * Dp / 2 : 0;
    k_step<<<npanel + nupd, 256, 0, s>>>(b, j, npanel, Linv, r, y, fail);
  }
  // column NT-1 has no sub-diagonal tiles, so no trailing update is left over
  if (b.NT > 0) k_band_back<<<1, kBackThreads, 0, s>>>(b, Linv, y, x);
}

}  // namespace dynohip
