// f16wave.h — the in-wave factorisation of a 16x16 FP64 block held in
// v_mfma_f64_16x16x4f64 accumulator layout (tilechol.hip's diagonal tiles and
// the small solve; tools/pivot_probe.hip times it in isolation).
#pragma once

#include <hip/hip_runtime.h>

namespace dynohip {

typedef double v4d __attribute__((ext_vector_type(4)));

// 1/sqrt(x): hardware estimate + two Newton steps (full FP64 accuracy)
__device__ __forceinline__ double rsqrt_nr(double x) {
  double y = __builtin_amdgcn_rsq(x);
  y = y * (1.5 - 0.5 * x * y * y);
  y = y * (1.5 - 0.5 * x * y * y);
  return y;
}

// 1/x: hardware estimate + two Newton steps (full FP64 accuracy); four
// dependent FMAs, half the chain of the reciprocal square root
__device__ __forceinline__ double rcp_nr(double x) {
  double y = __builtin_amdgcn_rcp(x);
  y = __builtin_fma(__builtin_fma(-x, y, 1.0), y, y);
  y = __builtin_fma(__builtin_fma(-x, y, 1.0), y, y);
  return y;
}

// ---- 16x16 in-wave factorisation (no barriers) --------------------------
// A 16x16 block in MFMA accumulator layout: lane l, register r holds
// element (row (l>>4) + 4r, column l&15). The same registers serve as the
// B operand of v_mfma_f64_16x16x4 for K-slice r, and as the A operand of
// the block's transpose.

__device__ __forceinline__ double bcast_row_lane(double v, int p) {
  // lane p of every 16-lane row -> the whole row (DPP row_newbcast)
  switch (p) {
// (every source lane exists, so no "old" value is needed: one v_mov_b64_dpp
// instead of a copy plus an in-place DPP move)
#define NB(q) case q: return __builtin_amdgcn_update_dpp(__builtin_nan(""), v, 0x150 + q, 0xf, 0xf, true);
    NB(0) NB(1) NB(2) NB(3) NB(4) NB(5) NB(6) NB(7) NB(8) NB(9) NB(10) NB(11) NB(12) NB(13) NB(14) NB(15)
#undef NB
  }
  return v;
}

// row group G (lanes 16G..16G+15) of v broadcast to all four row groups with
// the gfx950 lane swaps: permlane32_swap(v, v) gives [r0 r1 r0 r1] and
// [r2 r3 r2 r3], permlane16_swap of one of them with itself gives its two
// rows each broadcast. Four VALU swaps, no LDS round trip (ds_bpermute).
__device__ __forceinline__ unsigned row_bcast32(unsigned v, int G) {
  const auto a = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  const unsigned s = G < 2 ? a[0] : a[1];
  const auto b = __builtin_amdgcn_permlane16_swap(s, s, false, false);
  return (G & 1) ? b[1] : b[0];
}
__device__ __forceinline__ double row_bcast(double v, int G) {
  const unsigned lo = row_bcast32(static_cast<unsigned>(__double2loint(v)), G);
  const unsigned hi = row_bcast32(static_cast<unsigned>(__double2hiint(v)), G);
  return __hiloint2double(static_cast<int>(hi), static_cast<int>(lo));
}

__device__ __forceinline__ double pull_lane(double v, int src) {
  const int a = src << 2;
  const int lo = __builtin_amdgcn_ds_bpermute(a, __double2loint(v));
  const int hi = __builtin_amdgcn_ds_bpermute(a, __double2hiint(v));
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double read_lane(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

// B (symmetric, full) = U^T U; on return W = U^-1 (upper) and B is
// scratch. Right-looking by rows: pivot p's row is pulled across row
// groups (ds_bpermute), its column broadcast within them (DPP). Entries
// of B in rows or columns <= p are never read after pivot p, so the
// trailing update runs unmasked on the registers that still hold rows > p.
// W is updated unscaled (W~[c][i] -= W~[c][p] U[p][i] / U[p][p]) and each
// column is scaled by its 1/U[j][j] once at the end.
// dscr: 16 doubles of LDS scratch for the pivots. The column masks come from
// a per-lane counter made opaque every pivot, so the compiler cannot hoist
// sixteen of them into (spilled) scalar registers.
__device__ __forceinline__ void factor16_wave(v4d& B, v4d& W, int l, bool& ok, double* dscr) {
  const int j = l & 15;
  int jd = j;   // j - p at pivot p
#pragma unroll
  for (int p = 0; p < 16; ++p) {
    const int rp = p >> 2, gp = p & 3;
    const double d = read_lane(B[rp], 16 * gp + p);
    const double rowp = row_bcast(B[rp], gp);           // B[p][j]
    const double f = rowp * rcp_nr(d);                   // U[p][j] / U[p][p]
    asm volatile("" : "+v"(jd));
    const double fm = jd > 0 ? f : 0.0;
    jd -= 1;
    dscr[p] = d;   // every lane, same value

#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (4 * r + 3 > p) B[r] -= bcast_row_lane(B[r], p) * f;     // rows g+4r > p
      if (4 * r <= p) W[r] -= bcast_row_lane(W[r], p) * fm;      // W~[c][p] != 0 only for c <= p
    }
  }
  asm volatile("" ::: "memory");   // read back through LDS, not a 16-way select
  const double dj = dscr[j];   // this lane's column scale 1/U[j][j] = 1/sqrt(d_j)
  const double myrs = rsqrt_nr(dj);
#pragma unroll
  for (int r = 0; r < 4; ++r) W[r] *= myrs;
  // every pivot positive and finite (NaN fails both tests), checked once
  ok = ok && __all((dj > 0.0) && (dj < 1e300));
}


// ---- the same factorisation in four-pivot sub-blocks --------------------
// Sub-block s (pivots 4s..4s+3) is register s of the block: rows 4s+g of
// row group g. Its four rows are first replicated to every row group (three
// gfx950 lane swaps per dword), so that within the sub-block each pivot works
// on rows held in the lane itself: per pivot one DPP broadcast of the pivot,
// the reciprocal, the scaled row f_p = B[p][.] / d_p, and for each later row
// of the sub-block one DPP broadcast of its multiplier f_p[4s+k] and one FMA.
// The rows below the sub-block then take its rank-4 update in a single
// v_mfma_f64_16x16x4f64: B -= F^T R, F the sub-block's scaled rows (A
// operand, lane (k, m) = f_{4s+k}[m]) and R its rows at their pivot steps (B
// operand, lane (k, n) = R_k[n]), each selected by row group. W~ = L^-T is
// updated by columns as in factor16_wave; rows and columns of B at or above
// the sub-block are dead after it (never read), so no update is masked.
__device__ __forceinline__ void groups4_32(unsigned v, unsigned (&o)[4]) {
  const auto a = __builtin_amdgcn_permlane32_swap(v, v, false, false);    // [r0 r1 r0 r1], [r2 r3 r2 r3]
  const auto b = __builtin_amdgcn_permlane16_swap(a[0], a[0], false, false);
  const auto c = __builtin_amdgcn_permlane16_swap(a[1], a[1], false, false);
  o[0] = b[0];
  o[1] = b[1];
  o[2] = c[0];
  o[3] = c[1];
}
// o[k] = v of row group k (the lane's column), in every lane
__device__ __forceinline__ void groups4(double v, double (&o)[4]) {
  unsigned lo[4], hi[4];
  groups4_32(static_cast<unsigned>(__double2loint(v)), lo);
  groups4_32(static_cast<unsigned>(__double2hiint(v)), hi);
#pragma unroll
  for (int k = 0; k < 4; ++k) o[k] = __hiloint2double(static_cast<int>(hi[k]), static_cast<int>(lo[k]));
}
// x_g for the lane's row group g (values, not an array: a select between
// array elements is folded into a dynamically indexed load, which moves the
// array to LDS)
__device__ __forceinline__ double sel_group(double x0, double x1, double x2, double x3, bool g0, bool g1) {
  const double t0 = g0 ? x1 : x0;
  const double t1 = g0 ? x3 : x2;
  return g1 ? t1 : t0;
}

// 1/x from the hardware estimate y with one cubic step, y (1 + e + e^2),
// e = 1 - x y: three dependent FMAs where two Newton steps take four (the
// estimate's relative error cubed is far below the FP64 rounding)
__device__ __forceinline__ double rcp_cubic(double x) {
  const double y = __builtin_amdgcn_rcp(x);
  const double e = __builtin_fma(-x, y, 1.0);
  return __builtin_fma(y, __builtin_fma(e, e, e), y);
}

// v where (lane & 15) > P, else +0: the lane mask is a constant, set up by
// two scalar moves right here (not hoisted into a bank of SGPR masks) and
// applied by two v_cndmask
template <int P>
__device__ __forceinline__ double keep_cols_above(double v) {
  constexpr uint32_t row = (0xFFFFu << (P + 1)) & 0xFFFFu;
  constexpr uint32_t half = row | (row << 16);
  uint32_t mlo = half, mhi = half;
  asm volatile("" : "+s"(mlo), "+s"(mhi));
  const uint64_t m = (static_cast<uint64_t>(mhi) << 32) | mlo;
  int lo, hi;
  asm("v_cndmask_b32_e64 %0, 0, %2, %4\n\tv_cndmask_b32_e64 %1, 0, %3, %4"
      : "=&v"(lo), "=v"(hi)
      : "v"(__double2loint(v)), "v"(__double2hiint(v)), "s"(m));
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ void factor16_blk4(v4d& B, v4d& W, int l, bool& ok, double* dscr) {
  const int j = l & 15;
  const bool g0 = (l >> 4) & 1, g1 = (l >> 5) & 1;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    double R[4], F[4];
    groups4(B[s], R);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int p = 4 * s + c;
      const double d = bcast_row_lane(R[c], p);   // B[p][p] after pivots < p
      const double f = R[c] * rcp_cubic(d);       // U[p][j] / U[p][p]
      double fm;
      switch (p) {
#define KC(q) case q: fm = keep_cols_above<q>(f); break;
        KC(0) KC(1) KC(2) KC(3) KC(4) KC(5) KC(6) KC(7) KC(8) KC(9) KC(10) KC(11) KC(12) KC(13) KC(14) default: fm = 0.0;
#undef KC
      }
      dscr[p] = d;
      F[c] = f;
#pragma unroll
      for (int k = c + 1; k < 4; ++k) R[k] -= bcast_row_lane(f, 4 * s + k) * R[c];
#pragma unroll
      for (int r = 0; r <= s; ++r) W[r] -= bcast_row_lane(W[r], p) * fm;
    }
    if (s < 3)
      B = __builtin_amdgcn_mfma_f64_16x16x4f64(-sel_group(F[0], F[1], F[2], F[3], g0, g1),
                                               sel_group(R[0], R[1], R[2], R[3], g0, g1), B, 0, 0, 0);
  }
  asm volatile("" ::: "memory");   // read back through LDS, not a 16-way select
  const double dj = dscr[j];
  const double myrs = rsqrt_nr(dj);
#pragma unroll
  for (int r = 0; r < 4; ++r) W[r] *= myrs;
  ok = ok && __all((dj > 0.0) && (dj < 1e300));
}

// the form the kernels use (DYNOHIP_F16_PIVOT: the pivot-by-pivot form,
// for A/B measurements)
__device__ __forceinline__ void factor16(v4d& B, v4d& W, int l, bool& ok, double* dscr) {
#ifdef DYNOHIP_F16_PIVOT
  factor16_wave(B, W, l, ok, dscr);
#else
  factor16_blk4(B, W, l, ok, dscr);
#endif
}

}  // namespace dynohip
