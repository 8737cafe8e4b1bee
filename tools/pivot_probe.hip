// pivot_probe.hip — cycles per pivot of the in-wave 16x16 factorisation
// (tilechol.hip factor16_wave) in isolation: one wave factors a 16x16 SPD
// block `reps` times back to back, timed with s_memtime; W = U^-1 is written
// out so the host can check it (W^T B W = I). Built and run by
// tools/pivot_probe.py (hipcc, ctypes). Variants: 0 factor16_wave (pivot by
// pivot), 1 factor16_blk4 (the kernels' form), 2/3 the next pivot formed a
// step ahead (cubic / bare reciprocal), 4/5 the DPP broadcast folded into
// v_fmac_f64_dpp, 6 the sub-block's pivots from in-lane replicas
// (profiles/r05/pivot/probe_inlane.log: 189.5 against 171.5 cycles per pivot,
// bit-identical).
#include <hip/hip_runtime.h>

#include "../dynosam_amd/csrc/f16wave.h"

using namespace dynohip;

// experimental: factor16_blk4 with the next pivot formed one step ahead from
// three scalars (d_{p+1} = B[p+1][p+1] - f_p[p+1] B[p][p+1]), so the
// reciprocal chain runs beside the row updates; RCPN Newton-type steps
// (0: the bare estimate, 1: cubic)
template <int RCPN>
__device__ __forceinline__ double rcp_k(double x) {
  if constexpr (RCPN == 0) return __builtin_amdgcn_rcp(x);
  else return rcp_cubic(x);
}
template <int RCPN>
__device__ __forceinline__ void factor16_ahead(v4d& B, v4d& W, int l, bool& ok, double* dscr) {
  const int j = l & 15;
  const bool g0 = (l >> 4) & 1, g1 = (l >> 5) & 1;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    double R[4], F[4];
    groups4(B[s], R);
    double d = bcast_row_lane(R[0], 4 * s);
    double rc = rcp_k<RCPN>(d);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int p = 4 * s + c;
      const double f = R[c] * rc;                  // U[p][j] / U[p][p]
      double dn = 0.0, rn = 0.0;
      if (c < 3) {
        const double a = bcast_row_lane(R[c], p + 1), b = bcast_row_lane(R[c + 1], p + 1);
        dn = b - (a * rc) * a;                     // the next pivot from scalars
        rn = rcp_k<RCPN>(dn);
      }
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
      d = dn;
      rc = rn;
    }
    if (s < 3)
      B = __builtin_amdgcn_mfma_f64_16x16x4f64(-sel_group(F[0], F[1], F[2], F[3], g0, g1),
                                               sel_group(R[0], R[1], R[2], R[3], g0, g1), B, 0, 0, 0);
  }
  asm volatile("" ::: "memory");
  const double dj = dscr[j];
  const double myrs = rsqrt_nr(dj);
#pragma unroll
  for (int r = 0; r < 4; ++r) W[r] *= myrs;
  ok = ok && __all((dj > 0.0) && (dj < 1e300));
}

// acc -= bcast(src, lane P of each 16-lane row) * m in one instruction
// (v_fmac_f64 with a DPP row_newbcast source; the nop covers the VALU-write
// -> DPP-read hazard)
template <int P>
__device__ __forceinline__ void fmac_nb(double& acc, double src, double m) {
  asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
               : "+v"(acc)
               : "v"(src), "v"(m), "n"(P));
}
template <int RCPN>
__device__ __forceinline__ void factor16_fold(v4d& B, v4d& Wv, int l, bool& ok, double* dscr) {
  const int j = l & 15;
  double W[4] = {Wv[0], Wv[1], Wv[2], Wv[3]};
  const bool g0 = (l >> 4) & 1, g1 = (l >> 5) & 1;
#define FS(s)                                                                                    \
  {                                                                                              \
    double R[4], F[4];                                                                           \
    groups4(B[s], R);                                                                            \
    double d = bcast_row_lane(R[0], 4 * s);                                                      \
    double rc = rcp_k<RCPN>(d);                                                                  \
    FP(s, 0) FP(s, 1) FP(s, 2) FP(s, 3)                                                          \
    if (s < 3)                                                                                   \
      B = __builtin_amdgcn_mfma_f64_16x16x4f64(-sel_group(F[0], F[1], F[2], F[3], g0, g1),        \
                                               sel_group(R[0], R[1], R[2], R[3], g0, g1), B, 0, 0, 0); \
  }
#define FP(s, c)                                                                                 \
  {                                                                                              \
    constexpr int p = 4 * s + c;                                                                 \
    const double f = R[c] * rc;                                                                  \
    double dn = 0.0, rn = 0.0;                                                                   \
    if (c < 3) {                                                                                 \
      const double a = bcast_row_lane(R[c], p + 1), b = bcast_row_lane(R[c + 1], p + 1);         \
      dn = b - (a * rc) * a;                                                                     \
      rn = rcp_k<RCPN>(dn);                                                                      \
    }                                                                                            \
    const double fm = keep_cols_above<p < 15 ? p : 14>(f);                                      \
    dscr[p] = d;                                                                                 \
    F[c] = f;                                                                                    \
    if (c < 1) fmac_nb<4 * s + 1>(R[1], f, R[c]);                                                \
    if (c < 2) fmac_nb<4 * s + 2>(R[2], f, R[c]);                                                \
    if (c < 3) fmac_nb<4 * s + 3>(R[3], f, R[c]);                                                \
    if (p < 15) {                                                                                \
      fmac_nb<p>(W[0], W[0], fm);                                                                \
      if (s >= 1) fmac_nb<p>(W[1], W[1], fm);                                                    \
      if (s >= 2) fmac_nb<p>(W[2], W[2], fm);                                                    \
      if (s >= 3) fmac_nb<p>(W[3], W[3], fm);                                                    \
    }                                                                                            \
    d = dn;                                                                                      \
    rc = rn;                                                                                     \
  }
  FS(0) FS(1) FS(2) FS(3)
#undef FP
#undef FS
  asm volatile("" ::: "memory");
  const double dj = dscr[j];
  const double myrs = rsqrt_nr(dj);
#pragma unroll
  for (int r = 0; r < 4; ++r) Wv[r] = W[r] * myrs;
  ok = ok && __all((dj > 0.0) && (dj < 1e300));
}

// candidate: factor16_blk4 with each four-pivot sub-block's upper triangle
// replicated in every lane (ten DPP broadcasts up front), so the pivots,
// reciprocals and multipliers of the sub-block come from in-lane arithmetic
// (no DPP on the pivot chain); every replicated value is the same operation
// on the same operands as in the lane that owns its column, so W and the
// factor are factor16_blk4's bit for bit
__device__ __forceinline__ void factor16_inlane(v4d& B, v4d& W, int l, bool& ok, double* dscr) {
  const int j = l & 15;
  const bool g0 = (l >> 4) & 1, g1 = (l >> 5) & 1;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    double R[4], F[4], a[4][4];
    groups4(B[s], R);
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int d = c; d < 4; ++d) a[c][d] = bcast_row_lane(R[c], 4 * s + d);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int p = 4 * s + c;
      const double d = a[c][c];
      const double rc = rcp_cubic(d);
      const double f = R[c] * rc;
      double fm;
      switch (p) {
#define KC(q) case q: fm = keep_cols_above<q>(f); break;
        KC(0) KC(1) KC(2) KC(3) KC(4) KC(5) KC(6) KC(7) KC(8) KC(9) KC(10) KC(11) KC(12) KC(13) KC(14) default: fm = 0.0;
#undef KC
      }
      dscr[p] = d;
      F[c] = f;
#pragma unroll
      for (int k = c + 1; k < 4; ++k) {
        const double m = a[c][k] * rc;
        R[k] -= m * R[c];
#pragma unroll
        for (int e = k; e < 4; ++e) a[k][e] -= m * a[c][e];
      }
#pragma unroll
      for (int r = 0; r <= s; ++r) W[r] -= bcast_row_lane(W[r], p) * fm;
    }
    if (s < 3)
      B = __builtin_amdgcn_mfma_f64_16x16x4f64(-sel_group(F[0], F[1], F[2], F[3], g0, g1),
                                               sel_group(R[0], R[1], R[2], R[3], g0, g1), B, 0, 0, 0);
  }
  asm volatile("" ::: "memory");
  const double dj = dscr[j];
  const double myrs = rsqrt_nr(dj);
#pragma unroll
  for (int r = 0; r < 4; ++r) W[r] *= myrs;
  ok = ok && __all((dj > 0.0) && (dj < 1e300));
}

template <int V>
__global__ __launch_bounds__(64) void k_probe(const double* __restrict__ Bin, double* __restrict__ Wout,
                                              unsigned long long* __restrict__ cyc, int reps) {
  __shared__ double dscr[16];
  const int l = threadIdx.x;
  v4d B0;
#pragma unroll
  for (int r = 0; r < 4; ++r) B0[r] = Bin[((l >> 4) + 4 * r) * 16 + (l & 15)];
  v4d W;
  bool ok = true;
  unsigned long long t0 = 0, t1 = 0;
  for (int it = 0; it < reps; ++it) {
    v4d B = B0;
    asm volatile("" : "+v"(B));
#pragma unroll
    for (int r = 0; r < 4; ++r) W[r] = ((l >> 4) + 4 * r == (l & 15)) ? 1.0 : 0.0;
    if (it == 1) t0 = __builtin_amdgcn_s_memtime();
    if constexpr (V == 0) factor16_wave(B, W, l, ok, dscr);
    else if constexpr (V == 1) factor16_blk4(B, W, l, ok, dscr);
    else if constexpr (V == 2) factor16_ahead<1>(B, W, l, ok, dscr);
    else if constexpr (V == 3) factor16_ahead<0>(B, W, l, ok, dscr);
    else if constexpr (V == 4) factor16_fold<1>(B, W, l, ok, dscr);
    else if constexpr (V == 5) factor16_fold<0>(B, W, l, ok, dscr);
    else factor16_inlane(B, W, l, ok, dscr);
    asm volatile("" : "+v"(W));
  }
  t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int r = 0; r < 4; ++r) Wout[((l >> 4) + 4 * r) * 16 + (l & 15)] = W[r];
  if (l == 0) {
    cyc[0] = t1 - t0;
    cyc[1] = ok ? 1 : 0;
  }
}

__global__ void k_rcp(const double* __restrict__ x, double* __restrict__ y, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = __builtin_amdgcn_rcp(x[i]);
}

// the hardware reciprocal estimate (v_rcp_f64) of n doubles
extern "C" int probe_rcp(const double* xh, double* yh, int n) {
  double *x, *y;
  if (hipMalloc(&x, n * 8) || hipMalloc(&y, n * 8)) return -1;
  (void)hipMemcpy(x, xh, n * 8, hipMemcpyHostToDevice);
  k_rcp<<<(n + 255) / 256, 256>>>(x, y, n);
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  (void)hipMemcpy(yh, y, n * 8, hipMemcpyDeviceToHost);
  (void)hipFree(x);
  (void)hipFree(y);
  return 0;
}

extern "C" int probe_run(int variant, const double* Bh, double* Wh, unsigned long long* cyc, int reps) {
  double *B, *W;
  unsigned long long* c;
  if (hipMalloc(&B, 256 * 8) || hipMalloc(&W, 256 * 8) || hipMalloc(&c, 16)) return -1;
  (void)hipMemcpy(B, Bh, 256 * 8, hipMemcpyHostToDevice);
  if (variant == 0) k_probe<0><<<1, 64>>>(B, W, c, reps);
  else if (variant == 1) k_probe<1><<<1, 64>>>(B, W, c, reps);
  else if (variant == 2) k_probe<2><<<1, 64>>>(B, W, c, reps);
  else if (variant == 3) k_probe<3><<<1, 64>>>(B, W, c, reps);
  else if (variant == 4) k_probe<4><<<1, 64>>>(B, W, c, reps);
  else if (variant == 5) k_probe<5><<<1, 64>>>(B, W, c, reps);
  else k_probe<6><<<1, 64>>>(B, W, c, reps);
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  (void)hipMemcpy(Wh, W, 256 * 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(cyc, c, 16, hipMemcpyDeviceToHost);
  (void)hipFree(B);
  (void)hipFree(W);
  (void)hipFree(c);
  return 0;
}

typedef double d2v __attribute__((ext_vector_type(2)));

// f64 MFMA rate: cycles per v_mfma_f64_16x16x4f64 on one wave, (0) four
// independent accumulator chains fed from registers, (1) the same with the
// operands read from an LDS tile of row stride 68 doubles (as pend_block),
// (2) one dependent chain from registers, (3) as (1) with each lane's four
// k-steps of a 16-wide k-block consecutive (two 16-byte reads per operand),
// (4) / (5) as (3) with one / two accumulator chains
template <int V>
__global__ __launch_bounds__(64) void k_mfma_rate(const double* __restrict__ in, double* __restrict__ out,
                                                  unsigned long long* __restrict__ cyc, int reps) {
  __shared__ double P[64 * 68];
  const int l = threadIdx.x, li = l & 15, lk = l >> 4;
  for (int i = l; i < 64 * 68; i += 64) P[i] = in[i % 256];
  __syncthreads();
  v4d c[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) c[s] = v4d{0.0, 0.0, 0.0, 0.0};
  double a = in[l], b = in[64 + l];
  d2v qa0, qa1, qb0, qb1;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < reps; ++it) {
#pragma unroll
    for (int K = 0; K < 4; ++K)
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        if constexpr (V == 1) {
          a = -P[li * 68 + 16 * K + 4 * s4 + lk];
          b = P[(16 + li) * 68 + 16 * K + 4 * s4 + lk];
        }
        if constexpr (V >= 3) {   // lane lk takes the four consecutive k of its quarter: 16-byte reads
          if (s4 == 0) {
            const d2v* pa = reinterpret_cast<const d2v*>(P + li * 68 + 16 * K + 4 * lk);
            const d2v* pb = reinterpret_cast<const d2v*>(P + (16 + li) * 68 + 16 * K + 4 * lk);
            qa0 = pa[0]; qa1 = pa[1]; qb0 = pb[0]; qb1 = pb[1];
          }
          a = -(s4 < 2 ? qa0[s4] : qa1[s4 - 2]);
          b = s4 < 2 ? qb0[s4] : qb1[s4 - 2];
        }
        if constexpr (V == 2 || V == 4) c[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[0], 0, 0, 0);
        else if constexpr (V == 5) c[s4 & 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[s4 & 1], 0, 0, 0);
        else c[s4] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[s4], 0, 0, 0);
      }
    asm volatile("" : "+v"(a), "+v"(b));
  }
  v4d tot = (c[0] + c[1]) + (c[2] + c[3]);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int r = 0; r < 4; ++r) out[r * 64 + l] = tot[r];
  if (l == 0) cyc[0] = t1 - t0;
}

extern "C" int probe_mfma(int variant, const double* inh, unsigned long long* cyc, int reps) {
  double *in, *out;
  unsigned long long* c;
  if (hipMalloc(&in, 256 * 8) || hipMalloc(&out, 256 * 8) || hipMalloc(&c, 16)) return -1;
  (void)hipMemcpy(in, inh, 256 * 8, hipMemcpyHostToDevice);
  if (variant == 0) k_mfma_rate<0><<<1, 64>>>(in, out, c, reps);
  else if (variant == 1) k_mfma_rate<1><<<1, 64>>>(in, out, c, reps);
  else if (variant == 2) k_mfma_rate<2><<<1, 64>>>(in, out, c, reps);
  else if (variant == 3) k_mfma_rate<3><<<1, 64>>>(in, out, c, reps);
  else if (variant == 4) k_mfma_rate<4><<<1, 64>>>(in, out, c, reps);
  else k_mfma_rate<5><<<1, 64>>>(in, out, c, reps);
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  (void)hipMemcpy(cyc, c, 8, hipMemcpyDeviceToHost);
  (void)hipFree(in);
  (void)hipFree(out);
  (void)hipFree(c);
  return 0;
}
