// band.hip — block-banded Cholesky of the reduced (Schur) pose system and
// its triangular solves, 64x64 FP64 tiles, lower band stored by column tile.
//
// Per column tile j (stream-ordered launches, no inter-workgroup sync):
//   k_panel(j)   grid D_j+1: every workgroup factors the diagonal tile in
//                registers (right-looking, 4x4 sub-block per thread, one
//                barrier per pivot) and builds L_jj^-1 alongside; block 0
//                stores L_jj^-1 and y_j = L_jj^-1 r_j (forward substitution
//                fused into the factorisation); block d >= 1 turns tile
//                (j+d, j) into L(j+d, j) = A L_jj^-T (a GEMM with the
//                explicit inverse) and applies r_{j+d} -= L(j+d, j) y_j.
//   k_update(j)  grid D_j(D_j+1)/2: trailing tiles -= L(j+d1,j) L(j+d2,j)^T.
//   k_band_back  one workgroup: x_j = L_jj^-T (y_j - sum_d L(j+d,j)^T x_{j+d}).
// A non-positive pivot sets *fail (the LM treats the step as failed,
// GTSAM's IndeterminantLinearSystemException path).
#include <hip/hip_runtime.h>

#include "kernels.hpp"

namespace dynohip {

namespace {

constexpr int T = kTile;
constexpr int LD = T + 1;            // padded LDS row stride
constexpr int kPanelThreads = 320;  // 5 waves: 272 sub-block owners
constexpr int kSub = 16;             // 4x4 sub-blocks per tile side
constexpr int kLowerSub = kSub * (kSub + 1) / 2;  // 136

__device__ __forceinline__ void sub_index(int s, int& bi, int& bj) {
  int i = static_cast<int>((sqrtf(8.0f * s + 1.0f) - 1.0f) * 0.5f);
  while (i * (i + 1) / 2 > s) --i;
  while ((i + 1) * (i + 2) / 2 <= s) ++i;
  bi = i;
  bj = s - i * (i + 1) / 2;
}

// 64x64x64 GEMM on LDS operands: C[r][c] = sum_m A[r][m] * B[c][m]
// (B^T product), 4x4 outputs per thread for threads 0..255.
__device__ __forceinline__ void gemm_abt_4x4(const double* As, const double* Bs, int tid, double acc[4][4],
                                             int mmax = T) {
  const int r0 = (tid >> 4) * 4, c0 = (tid & 15) * 4;
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int w = 0; w < 4; ++w) acc[u][w] = 0.0;
  for (int m = 0; m < mmax; ++m) {
    double a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a[u] = As[(r0 + u) * LD + m];
      b[u] = Bs[(c0 + u) * LD + m];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int w = 0; w < 4; ++w) acc[u][w] += a[u] * b[w];
  }
}

__device__ __forceinline__ void load_tile_lds(const double* __restrict__ src, double* dst, int tid, int nthreads) {
  const double2* s2 = reinterpret_cast<const double2*>(src);
  for (int e = tid; e < T * T / 2; e += nthreads) {
    const double2 v = s2[e];
    const int r = (2 * e) / T, c = (2 * e) % T;
    dst[r * LD + c] = v.x;
    dst[r * LD + c + 1] = v.y;
  }
}

__global__ __launch_bounds__(kPanelThreads) void k_panel(BandDev b, int j, double* __restrict__ Linv,
                                                         double* __restrict__ r, double* __restrict__ y,
                                                         int* fail) {
  __shared__ double As[T * LD];
  __shared__ double Xs[T * LD];
  __shared__ double colbuf[2][T];
  __shared__ double rowbuf[2][T];
  __shared__ double akkbuf[2];
  __shared__ double yv[T];
  const int tid = threadIdx.x;
  const int d = blockIdx.x;
  const double* diag = b.band + b.off[j];
  if (d > 0) load_tile_lds(diag + static_cast<int64_t>(d) * T * T, As, tid, kPanelThreads);
  // ---- roles: 136 threads own 4x4 sub-blocks of A (lower), 136 of the inverse
  const bool isA = tid < kLowerSub;
  const bool isX = tid >= kLowerSub && tid < 2 * kLowerSub;
  int bi = 0, bj = 0;
  if (isA) sub_index(tid, bi, bj);
  if (isX) sub_index(tid - kLowerSub, bi, bj);
  double v[4][4];
  if (isA) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const double4 q = *reinterpret_cast<const double4*>(diag + (4 * bi + u) * T + 4 * bj);
      v[u][0] = q.x; v[u][1] = q.y; v[u][2] = q.z; v[u][3] = q.w;
    }
  } else {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int w = 0; w < 4; ++w) v[u][w] = (isX && bi == bj && u == w) ? 1.0 : 0.0;
  }
  // Right-looking elimination of A and forward elimination of [A | I]:
  // at pivot k, with c_i = a_ik (i > k, else 0), r_c = acc_kc (row k of the
  // running inverse, exactly 0 for c > k):
  //   a_ij  -= c_i c_j / a_kk        (i, j > k; lower part kept)
  //   acc_ic -= c_i r_c / a_kk       (i > k)
  //   acc_kc *= 1 / sqrt(a_kk)       (row k of L^-1 is final)
  // Publishers write exact zeros where a row / column is inactive, so every
  // update below is unconditional (no per-element branches).
  bool bad = false;
#ifndef DH_NO_PIVOT
  for (int kb = 0; kb < kSub; ++kb) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int k = 4 * kb + kk, p = kk & 1;
      if (isA && bj == kb) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int i = 4 * bi + u;
          colbuf[p][i] = i > k ? v[u][kk] : 0.0;
          if (i == k) akkbuf[p] = v[u][kk];
        }
      }
      if (isX && bi == kb) {
#pragma unroll
        for (int w = 0; w < 4; ++w) rowbuf[p][4 * bj + w] = v[kk][w];
      }
      __syncthreads();
      double akk = akkbuf[p];
      if (!(akk > 0.0) || !isfinite(akk)) {
        bad = true;
        akk = 1.0;
      }
#ifdef DH_FAST_RCP
      double rinv = __builtin_amdgcn_rcp(akk);
      rinv = rinv * (2.0 - akk * rinv);
      rinv = rinv * (2.0 - akk * rinv);
#else
      const double rinv = 1.0 / akk;
#endif
      if (isA && bj >= kb) {
        double ci[4], cj[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          ci[u] = colbuf[p][4 * bi + u] * rinv;
          cj[u] = colbuf[p][4 * bj + u];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int w = 0; w < 4; ++w) v[u][w] -= ci[u] * cj[w];
      }
      if (isX && bi >= kb && bj <= kb) {
        double ci[4], rc[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          ci[u] = colbuf[p][4 * bi + u] * rinv;
          rc[u] = rowbuf[p][4 * bj + u];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int w = 0; w < 4; ++w) v[u][w] -= ci[u] * rc[w];
        if (bi == kb) {
          const double isq = sqrt(rinv);
#pragma unroll
          for (int w = 0; w < 4; ++w) v[kk][w] *= isq;
        }
      }
    }
  }
#endif
  if (bad && tid == 0 && d == 0) *fail = 1;
  __syncthreads();
  // inverse -> LDS (full square, upper zero) ; block 0 also -> global
  if (isX) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        Xs[(4 * bi + u) * LD + 4 * bj + w] = v[u][w];
        if (bi != bj) Xs[(4 * bj + w) * LD + 4 * bi + u] = 0.0;
      }
  }
  __syncthreads();
  if (d == 0) {
    double* dst = Linv + static_cast<int64_t>(j) * T * T;
    for (int e = tid; e < T * T; e += kPanelThreads) dst[e] = Xs[(e / T) * LD + e % T];
  }
  // y_j = L_jj^-1 r_j (every block; block 0 stores it)
  const double* rj = r + static_cast<int64_t>(j) * T;
  if (tid < T) {
    double s = 0.0;
    for (int m = 0; m <= tid; ++m) s += Xs[tid * LD + m] * rj[m];
    yv[tid] = s;
    if (d == 0) y[static_cast<int64_t>(j) * T + tid] = s;
  }
  if (d == 0) return;
  __syncthreads();
  // L(j+d, j) = A L^-T  (Xs holds L^-1: C[r][c] = sum_m A[r][m] Linv[c][m])
  double acc[4][4];
  if (tid < 256) {
    gemm_abt_4x4(As, Xs, tid, acc);
    const int r0 = (tid >> 4) * 4, c0 = (tid & 15) * 4;
    double* dst = b.band + b.off[j] + static_cast<int64_t>(d) * T * T;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      *reinterpret_cast<double4*>(dst + (r0 + u) * T + c0) = make_double4(acc[u][0], acc[u][1], acc[u][2], acc[u][3]);
    }
  }
  __syncthreads();  // all reads of As done before reuse
  if (tid < 256) {
    const int r0 = (tid >> 4) * 4, c0 = (tid & 15) * 4;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int w = 0; w < 4; ++w) As[(r0 + u) * LD + c0 + w] = acc[u][w];
  }
  __syncthreads();
  // r_{j+d} -= L(j+d, j) y_j
  if (tid < T) {
    double s = 0.0;
    for (int m = 0; m < T; ++m) s += As[tid * LD + m] * yv[m];
    r[static_cast<int64_t>(j + d) * T + tid] -= s;
  }
}

// trailing update of column j: tile(j+d1, j+d2) -= L(j+d1,j) L(j+d2,j)^T
__global__ __launch_bounds__(256) void k_update(BandDev b, int j) {
  __shared__ double As[T * LD];
  __shared__ double Bs[T * LD];
  int t = blockIdx.x, d1 = 1;
  while (t >= d1) { t -= d1; ++d1; }
  const int d2 = t + 1;
  const double* A = b.band + b.off[j] + static_cast<int64_t>(d1) * T * T;
  const double* B = b.band + b.off[j] + static_cast<int64_t>(d2) * T * T;
  double* C = b.band + b.off[j + d2] + static_cast<int64_t>(d1 - d2) * T * T;
  const int tid = threadIdx.x;
  load_tile_lds(A, As, tid, 256);
  load_tile_lds(B, Bs, tid, 256);
  __syncthreads();
  double acc[4][4];
  gemm_abt_4x4(As, Bs, tid, acc);
  const int r0 = (tid >> 4) * 4, c0 = (tid & 15) * 4;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    double4* pc = reinterpret_cast<double4*>(C + (r0 + u) * T + c0);
    double4 q = *pc;
    q.x -= acc[u][0]; q.y -= acc[u][1]; q.z -= acc[u][2]; q.w -= acc[u][3];
    *pc = q;
  }
}

// backward substitution with the stored inverses (one workgroup)
constexpr int kBackThreads = 1024;
__global__ __launch_bounds__(kBackThreads) void k_band_back(BandDev b, const double* __restrict__ Linv,
                                                            const double* __restrict__ y, double* __restrict__ x) {
  __shared__ double part[kBackThreads / T][T];
  __shared__ double rv[T];
  const int tid = threadIdx.x, c = tid & (T - 1), q = tid >> 6;  // 16 parts
  constexpr int NP = kBackThreads / T;
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
    const int D = host_D[j];
    k_panel<<<D + 1, kPanelThreads, 0, s>>>(b, j, Linv, r, y, fail);
#ifndef DH_NO_UPDATE
    if (D > 0) k_update<<<D * (D + 1) / 2, 256, 0, s>>>(b, j);
#endif
  }
  if (b.NT > 0) k_band_back<<<1, kBackThreads, 0, s>>>(b, Linv, y, x);
}

}  // namespace dynohip
