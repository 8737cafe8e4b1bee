// tilechol.hip — Cholesky of the reduced (Schur) pose system as a DAG of
// 64x64 FP64 tile tasks (schedule built on the host, tiles.cpp), with the
// forward substitution fused in and a level-scheduled backward substitution.
//
// k_tasks runs one level of the schedule: every workgroup executes one task.
//   panel(k, i)   applies the last outstanding update of A(k,k) (L(k,c)
//       L(k,c)^T, into the accumulators) and of its own tile A(i,k). It then
//       factors the diagonal tile in registers (4x4-blocked right-looking
//       Cholesky on v_mfma_f64_16x16x4f64, one barrier per 4 pivots)
//       together with L_kk^-1, and computes y_k = L_kk^-1 r_k. Then
//         i == k: store L_kk^-1 and y_k;
//         i != k: L(i,k) = A(i,k) L_kk^-T (MFMA GEMM with the explicit
//                 inverse), r_i -= L(i,k) y_k.
//   update        A(i,j) -= L(i,c) L(j,c)^T (MFMA GEMM).
// The host schedule guarantees that no workgroup of a level writes what
// another workgroup of the same level reads or writes. Every tile receives
// its updates in a fixed order, so results are deterministic. k_back runs
// one level of x_k = L_kk^-T (y_k - sum_i L(i,k)^T x_i).
// A non-positive pivot sets *fail. The LM then treats the step as failed,
// like GTSAM's IndeterminantLinearSystemException path.
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
__device__ __forceinline__ void zero_acc(v4d acc[2][2]) {
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = v4d{0.0, 0.0, 0.0, 0.0};
}

// acc += A B^T
__device__ __forceinline__ void mfma_abt_acc(const double* As, const double* Bs, int wave, int lane, v4d acc[2][2]) {
  const int i0 = 32 * (wave >> 1), j0 = 32 * (wave & 1);
  const int li = lane & 15, lk = lane >> 4;
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

__device__ __forceinline__ void mfma_abt(const double* As, const double* Bs, int wave, int lane, v4d acc[2][2]) {
  zero_acc(acc);
  mfma_abt_acc(As, Bs, wave, lane, acc);
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

__device__ __forceinline__ double* slot_ptr(const TileDev& b, int32_t slot) {
  return b.slots + static_cast<int64_t>(slot) * T * T;
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

// sum over operand pairs [beg, end) of A B^T into acc (operands staged in
// Qs / Rs; a pair with A == B is loaded once)
__device__ __forceinline__ void sum_pairs(const TileDev& b, const int32_t* __restrict__ pairs, int beg, int end,
                                          double* Qs, double* Rs, int tid, int w, int l, v4d acc[2][2]) {
  zero_acc(acc);
  for (int e = beg; e < end; ++e) {
    const int32_t pa = pairs[2 * e], pb = pairs[2 * e + 1];
    __syncthreads();
    load_tile_lds(slot_ptr(b, pa), Qs, tid, 256);
    if (pb != pa) load_tile_lds(slot_ptr(b, pb), Rs, tid, 256);
    __syncthreads();
    mfma_abt_acc(Qs, pb != pa ? Rs : Qs, w, l, acc);
  }
}

__global__ __launch_bounds__(256) void k_tasks(TileDev b, const TileTask* __restrict__ tasks,
                                               const int32_t* __restrict__ pairs, double* __restrict__ Linv,
                                               const double* __restrict__ r, double* __restrict__ contrib,
                                               double* __restrict__ y, int* fail) {
  __shared__ double Ps[T * LD];   // pending diagonal operand L(k, c) -> later L_kk^-1
  __shared__ double Qs[T * LD];   // pair operand A
  __shared__ double Rs[T * LD];   // pair operand B
  __shared__ double As[T * LD];   // own tile (i, k)
  __shared__ double Pcol[2 * T * 4];
  __shared__ double Xrow[2 * 4 * T];
  __shared__ double vv[T];
  const TileTask tk = tasks[blockIdx.x];
  const int tid = threadIdx.x;
  const int w = tid >> 6, l = tid & 63;
  if (tk.kind == 1) {
    // ---- update: dst -= sum A B^T
    v4d acc[2][2];
    sum_pairs(b, pairs, tk.po_beg, tk.po_end, Qs, Rs, tid, w, l, acc);
    double* dst = slot_ptr(b, tk.dst);
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < 2; ++tj)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) dst[MFMA_ROW(w, l, ti, rr) * T + MFMA_COL(w, l, tj)] -= acc[ti][tj][rr];
    return;
  }
  // ---- panel
  const bool own = tk.i != tk.k;
  if (own) {
    // A(i,k) -= sum L(i,c) L(k,c)^T  (pending contributions)
    load_tile_lds(slot_ptr(b, tk.dst), As, tid, 256);
    if (tk.po_end > tk.po_beg) {
      v4d acc[2][2];
      sum_pairs(b, pairs, tk.po_beg, tk.po_end, Qs, Rs, tid, w, l, acc);
#pragma unroll
      for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) As[MFMA_ROW(w, l, ti, rr) * LD + MFMA_COL(w, l, tj)] -= acc[ti][tj][rr];
    }
  }
  v4d accA[4], accX[4];
  const double* diag = slot_ptr(b, tk.diag);
#pragma unroll
  for (int TJ = 0; TJ < 4; ++TJ)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = ACC_ROW(w, l, rr), col = ACC_COL(TJ, l);
      accA[TJ][rr] = diag[row * T + col];
      accX[TJ][rr] = row == col ? 1.0 : 0.0;
    }
  const int li = l & 15, lk = l >> 4;
  for (int e = tk.pd_beg; e < tk.pd_end; ++e) {
    // A_kk -= L(k,c) L(k,c)^T into the accumulators (K = 64)
    __syncthreads();
    load_tile_lds(slot_ptr(b, pairs[2 * e]), Ps, tid, 256);
    __syncthreads();
#pragma unroll 4
    for (int k0 = 0; k0 < T; k0 += 4) {
      const double a = -Ps[(16 * w + li) * LD + k0 + lk];
#pragma unroll
      for (int TJ = 0; TJ < 4; ++TJ)
        accA[TJ] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Ps[(16 * TJ + li) * LD + k0 + lk], accA[TJ], 0, 0, 0);
    }
  }
  __syncthreads();
  const bool ok = factor_tile_mfma(accA, accX, w, l, Pcol, Xrow);
  if (!ok && !own && tid == 0) *fail = 1;
  // L_kk^-1 -> Ps (full square; upper part is exactly zero)
#pragma unroll
  for (int TJ = 0; TJ < 4; ++TJ)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) Ps[ACC_ROW(w, l, rr) * LD + ACC_COL(TJ, l)] = accX[TJ][rr];
  if (!own) {
    double* dst = Linv + static_cast<int64_t>(tk.k) * T * T;
#pragma unroll
    for (int TJ = 0; TJ < 4; ++TJ)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) dst[ACC_ROW(w, l, rr) * T + ACC_COL(TJ, l)] = accX[TJ][rr];
  }
  // r_k minus the contributions L(k,c) y_c of the columns already eliminated
  if (tid < T) {
    double v = r[static_cast<int64_t>(tk.k) * T + tid];
    for (int e = b.row_start[tk.k]; e < b.row_start[tk.k + 1]; ++e)
      if (b.row_col[e] != tk.k) v -= contrib[static_cast<int64_t>(b.row_slot[e]) * T + tid];
    vv[tid] = v;
  }
  __syncthreads();
  // y_k = L_kk^-1 r_k
  const double yrow = lower_gemv4(Ps, vv, tid);
  __syncthreads();
  if ((tid & 3) == 0) {
    vv[tid >> 2] = yrow;
    if (!own) y[static_cast<int64_t>(tk.k) * T + (tid >> 2)] = yrow;
  }
  if (!own) return;
  // L(i, k) = A L^-T
  v4d acc[2][2];
  mfma_abt(As, Ps, w, l, acc);
  __syncthreads();
  double* dst = slot_ptr(b, tk.dst);
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
  // contribution of this tile to row i's right-hand side: L(i, k) y_k
  {
    const int row = tid >> 2, part = tid & 3;
    double s = 0.0;
    for (int m = part; m < T; m += 4) s += As[row * LD + m] * vv[m];
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    if (part == 0) contrib[static_cast<int64_t>(tk.dst) * T + row] = s;
  }
}

// one level of the backward substitution: a workgroup per column tile k,
// x_k = L_kk^-T (y_k - sum_i L(i,k)^T x_i)
__global__ __launch_bounds__(256) void k_back(TileDev b, const BackTask* __restrict__ tasks,
                                              const int32_t* __restrict__ ent, const double* __restrict__ Linv,
                                              const double* __restrict__ y, double* __restrict__ x) {
  constexpr int NP = 4;
  __shared__ double part[NP][T];
  __shared__ double rv[T];
  const BackTask tk = tasks[blockIdx.x];
  const int tid = threadIdx.x, c = tid & (T - 1), q = tid >> 6;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  for (int e = tk.beg; e < tk.end; ++e) {
    const double* L = slot_ptr(b, ent[2 * e]);
    const double* xi = x + static_cast<int64_t>(ent[2 * e + 1]) * T;
    // rows m = q, q+4, ...: 4 independent accumulators
    for (int m = q; m < T; m += 4 * NP) {
      s0 += L[m * T + c] * xi[m];
      s1 += L[(m + NP) * T + c] * xi[m + NP];
      s2 += L[(m + 2 * NP) * T + c] * xi[m + 2 * NP];
      s3 += L[(m + 3 * NP) * T + c] * xi[m + 3 * NP];
    }
  }
  part[q][c] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (tid < T) rv[tid] = y[static_cast<int64_t>(tk.k) * T + tid] - ((part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid]));
  __syncthreads();
  // x_k[c] = sum_{m >= c} Linv[m][c] rv[m]
  const double* Li = Linv + static_cast<int64_t>(tk.k) * T * T;
  double t = 0.0;
  for (int m = q; m < T; m += NP)
    if (m >= c) t += Li[m * T + c] * rv[m];
  part[q][c] = t;
  __syncthreads();
  if (tid < T)
    x[static_cast<int64_t>(tk.k) * T + tid] = (part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid]);
}

}  // namespace

void launch_tile_cholesky_solve(const TileDev& b, const TileSchedDev& sd, const std::vector<int32_t>& flevel,
                                const std::vector<int32_t>& blevel, double* Linv, const double* r, double* contrib,
                                double* y, double* x, int* fail, hipStream_t s) {
  for (size_t lv = 0; lv + 1 < flevel.size(); ++lv) {
    const int n = flevel[lv + 1] - flevel[lv];
    if (n > 0) k_tasks<<<n, 256, 0, s>>>(b, sd.ftask + flevel[lv], sd.pairs, Linv, r, contrib, y, fail);
  }
  for (size_t lv = 0; lv + 1 < blevel.size(); ++lv) {
    const int n = blevel[lv + 1] - blevel[lv];
    if (n > 0) k_back<<<n, 256, 0, s>>>(b, sd.btask + blevel[lv], sd.bent, Linv, y, x);
  }
}

}  // namespace dynohip
