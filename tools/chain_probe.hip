// Development probe (round 2, not used by the product): a "chain"
// factorisation of a 64x64 diagonal tile
// (factor_tile_chain + inverse_column, tilechol.hip) against the blocked
// 4-wave version (factor_tile_blk): cycles and max error of L^-1 against a
// host Cholesky inverse; plus the in-wave 16x16 pivot loops and the
// row-group broadcast.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/chain_probe.hip -o tools/chain_probe
#include "../dynosam_amd/csrc/tilechol.hip"

#include <cmath>
#include <cstdio>
#include <random>
#include <type_traits>
#include <vector>

namespace dynohip {
namespace {
// ---- the chain factorisation (one wave walks the pivot chain) -----------
// Row group G (lanes 16G..16G+15) of v, replicated into all four row
// groups, with two gfx950 lane swaps per dword instead of an LDS
// round trip: permlane16_swap(v, v) yields [R0,R0,R2,R2] (vdst) and
// [R1,R1,R3,R3] (src); permlane32_swap(x, x) of such an [Ra,Ra,Rb,Rb]
// yields [Ra,Ra,Ra,Ra] (vdst) and [Rb,Rb,Rb,Rb] (src).
__device__ __forceinline__ int bcast_group_b32(int v, int g) {
  const auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  const int x = (g & 1) ? static_cast<int>(a[1]) : static_cast<int>(a[0]);
  const auto b = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return (g & 2) ? static_cast<int>(b[1]) : static_cast<int>(b[0]);
}
__device__ __forceinline__ double bcast_group(double v, int g) {
  const int lo = bcast_group_b32(__double2loint(v), g);
  const int hi = bcast_group_b32(__double2hiint(v), g);
  return __hiloint2double(hi, lo);
}

// 1/x: hardware estimate + two Newton steps (full FP64 accuracy)
__device__ __forceinline__ double rcp_nr(double x) {
  double y = __builtin_amdgcn_rcp(x);
  double e = __builtin_fma(-x, y, 1.0);
  y = __builtin_fma(y, e, y);
  e = __builtin_fma(-x, y, 1.0);
  return __builtin_fma(y, e, y);
}

// compile-time loop: f(std::integral_constant<int, i>) for i in [B, E)
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// v += bcast_row_lane(v, P) * f as one v_fmac_f64 with a row_newbcast DPP
// source (the compiler does not fold the broadcast into the fmac itself).
// s_nop 1 covers the VALU-write -> DPP-read hazard, which the compiler does
// not see inside inline asm.
template <int P>
__device__ __forceinline__ double fmac_bcast(double v, double f) {
  asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
               : "+v"(v)
               : "v"(f), "n"(P));
  return v;
}

// factor16_wave with a shorter pivot chain: the pivot row comes from two
// lane swaps, the pivot itself by DPP from that row, and only 1/d is on the
// chain (the column scales 1/sqrt(d) of W are taken once at the end).
// hook(integral_constant<p>) runs at every pivot: MFMA work of the caller
// that overlaps the VALU chain.
struct NoPivotHook {
  template <class P>
  __device__ void operator()(P) const {}
};
template <class Hook = NoPivotHook>
__device__ __forceinline__ void factor16_chain(v4d& B, v4d& W, int l, bool& ok, Hook&& hook = Hook()) {
  const int j = l & 15;
  double mydiag = 1.0;
  bool good = true;
  static_for<0, 16>([&](auto pc) {
    constexpr int p = decltype(pc)::value;
    constexpr int rp = p >> 2, gp = p & 3;
    const double rowp = bcast_group(B[rp], gp);   // B[p][j]
    const double d = bcast_row_lane(rowp, p);      // B[p][p]
    good = good && (d > 0.0) && (d < 1e300);
    const double nf = rowp * -rcp_nr(d);           // -U[p][j] / U[p][p]
    const double nfm = j > p ? nf : 0.0;
    mydiag = j == p ? d : mydiag;
    hook(pc);
    // B += bcast(B) * nf in fmac form, so the DPP broadcast folds into
    // v_fmac_f64_dpp (no separate move)
    static_for<0, 4>([&](auto rc) {
      constexpr int r = decltype(rc)::value;
      if constexpr (4 * r + 3 > p) B[r] = fmac_bcast<p>(B[r], nf);
      if constexpr (4 * r <= p) W[r] = fmac_bcast<p>(W[r], nfm);
    });
  });
  const double rs = rsqrt_nr(mydiag);
#pragma unroll
  for (int r = 0; r < 4; ++r) W[r] *= rs;
  ok = ok && good;
}

// one 16x16x4 slice r of acc (+/-)= Y^T Z (blocks in accumulator layout)
__device__ __forceinline__ v4d mfma_tn_slice(const v4d& Y, const v4d& Z, v4d acc, int r, bool neg) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(neg ? -Y[r] : Y[r], Z[r], acc, 0, 0, 0);
}

__device__ __forceinline__ v4d ident16(int l) {
  v4d e;
#pragma unroll
  for (int r = 0; r < 4; ++r) e[r] = ((l >> 4) + 4 * r == (l & 15)) ? 1.0 : 0.0;
  return e;
}

// LDS of the chain factorisation: W_K (4 blocks), U_{K,J} (6 blocks, K < J),
// one block each in accumulator order (element r*64 + lane), and the step
// counter the chain wave raises after publishing step K.
struct ChainXch {
  double W[4][256];
  double U[6][256];
  int step;
};
constexpr int uidx(int K, int J) { return K == 0 ? J - 1 : (K == 1 ? J + 1 : 5); }
constexpr int bidx(int I, int J) { return I == 0 ? J : (I == 1 ? 3 + J : (I == 2 ? 5 + J : 9)); }

__device__ __forceinline__ void put_blk(double* d, const v4d& v, int l) {
#pragma unroll
  for (int r = 0; r < 4; ++r) d[r * 64 + l] = v[r];
}
__device__ __forceinline__ v4d get_blk(const double* d, int l) {
  v4d v;
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = d[r * 64 + l];
  return v;
}
__device__ __forceinline__ void chain_publish(ChainXch& x, int step) {
  __hip_atomic_store(&x.step, step, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void chain_wait(ChainXch& x, int step) {
  while (__hip_atomic_load(&x.step, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < step) __builtin_amdgcn_s_sleep(1);
}

// The ops step KP of the chain defers into the pivots of step KP+1, as
// 16x16x4 slices in dependency order: kind 0 = slice r of U_{KP,J} =
// W_KP^T A_{KP,J} (J >= KP+2), kind 1 = slice r of A_{I,J} -= U_{KP,I}^T
// U_{KP,J} (KP < I <= J, except the chain's own (KP+1, KP+1)); kind -1 = none.
struct DefOp {
  int kind, I, J, r;
};
constexpr DefOp def_op(int KP, int op) {
  int o = 0;
  for (int J = KP + 2; J < 4; ++J)
    for (int r = 0; r < 4; ++r, ++o)
      if (o == op) return DefOp{0, KP, J, r};
  for (int I = KP + 1; I < 4; ++I)
    for (int J = I; J < 4; ++J)
      if (!(I == KP + 1 && J == KP + 1))
        for (int r = 0; r < 4; ++r, ++o)
          if (o == op) return DefOp{1, I, J, r};
  return DefOp{-1, 0, 0, 0};
}
constexpr int def_count(int KP) {
  int n = 0;
  while (def_op(KP, n).kind >= 0) ++n;
  return n;
}

// Chain wave (wave 0): the right-looking blocked Cholesky A = U^T U of the
// 64x64 tile held as its 10 upper 16x16 blocks a[bidx(I, J)] (I <= J, full
// symmetric input). Step K factors block (K, K) in-wave, forms U_{K,K+1} and
// applies it to block (K+1, K+1) at once; the rest of step K (the other U
// blocks of row K and the trailing updates) is deferred into the pivots of
// step K+1's in-wave factorisation (def_op, two slices per pivot), where the
// matrix pipe is otherwise idle. W_K and the U blocks go to LDS for the
// inverse waves: x.step = K+1 once W_K, U_{K,K+1} and every U_{m,J} with
// m < K are published.
template <int HOOKS = 1>
__device__ __forceinline__ bool factor_tile_chain(v4d (&a)[10], ChainXch& x, int l, long long* stamps = nullptr) {
  bool ok = true;
  v4d u[4], Wp = v4d{0.0, 0.0, 0.0, 0.0};
  static_for<0, 4>([&](auto kc) {
    constexpr int K = decltype(kc)::value;
    v4d Wk = ident16(l);
    auto hook = [&](auto pc) {
      constexpr int P = decltype(pc)::value;
      if constexpr (K >= 1) {
        static_for<0, 2>([&](auto qc) {
          constexpr DefOp o = def_op(K - 1, 2 * P + decltype(qc)::value);
          if constexpr (o.kind == 0) {
            if constexpr (o.r == 0) u[o.J] = v4d{0.0, 0.0, 0.0, 0.0};
            u[o.J] = mfma_tn_slice(Wp, a[bidx(o.I, o.J)], u[o.J], o.r, false);
          } else if constexpr (o.kind == 1) {
            a[bidx(o.I, o.J)] = mfma_tn_slice(u[o.I], u[o.J], a[bidx(o.I, o.J)], o.r, true);
          }
        });
      }
    };
    static_assert(K == 0 || def_count(K - 1) <= 32, "deferred ops exceed the pivot slots");
    if constexpr (HOOKS == 1) {
      factor16_chain(a[bidx(K, K)], Wk, l, ok, hook);
    } else if constexpr (HOOKS == 2) {
      factor16_chain(a[bidx(K, K)], Wk, l, ok);   // timing ablation: deferred ops skipped
    } else {
      static_for<0, 16>([&](auto pc) { hook(pc); });
      factor16_chain(a[bidx(K, K)], Wk, l, ok);
    }
    if (stamps) stamps[2 * K] = clock64();
    if constexpr (K >= 1) {
      // the deferred U row of step K-1, computed during the pivots
      static_for<K + 1, 4>([&](auto jc) {
        constexpr int J = decltype(jc)::value;
        put_blk(x.U[uidx(K - 1, J)], u[J], l);
      });
    }
    put_blk(x.W[K], Wk, l);
    if constexpr (K < 3) {
      v4d un = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int r = 0; r < 4; ++r) un = mfma_tn_slice(Wk, a[bidx(K, K + 1)], un, r, false);
      u[K + 1] = un;
#pragma unroll
      for (int r = 0; r < 4; ++r) a[bidx(K + 1, K + 1)] = mfma_tn_slice(un, un, a[bidx(K + 1, K + 1)], r, true);
      put_blk(x.U[uidx(K, K + 1)], un, l);
    }
    chain_publish(x, K + 1);
    if (stamps) stamps[2 * K + 1] = clock64();
    Wp = Wk;
  });
  return ok;
}

// Inverse wave for block column j of X = L^-1 (L = U^T):
//   X_jj = W_j^T,  X_ij = -W_i^T sum_{m=j}^{i-1} U_{m,i}^T X_mj  (i > j).
// U_{m,i} (m < i) is published by step i of the chain (x.step >= i), W_i by
// step i+1. Writes X_ij (i >= j) into dst (row stride ld) and zeros above.
__device__ __forceinline__ void inverse_column(ChainXch& x, int j, int l, double* dst, int ld) {
  v4d X[4];
  chain_wait(x, j + 1);
  {
    const v4d Wj = get_blk(x.W[j], l), e = ident16(l);
    v4d z = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int r = 0; r < 4; ++r) z = mfma_tn_slice(Wj, e, z, r, false);
    X[j] = z;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i <= j) continue;
    chain_wait(x, i);
    v4d S = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      if (m < j || m >= i) continue;
      const v4d Um = get_blk(x.U[uidx(m, i)], l);
#pragma unroll
      for (int r = 0; r < 4; ++r) S = mfma_tn_slice(Um, X[m], S, r, false);
    }
    chain_wait(x, i + 1);
    const v4d Wi = get_blk(x.W[i], l);
    v4d z = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int r = 0; r < 4; ++r) z = mfma_tn_slice(Wi, S, z, r, true);
    X[i] = z;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * i + (l >> 4) + 4 * r, col = 16 * j + (l & 15);
      dst[row * ld + col] = i >= j ? X[i][r] : 0.0;
    }
}

}  // namespace
}  // namespace dynohip

using namespace dynohip;

__global__ __launch_bounds__(64) void k_bcast(int* out) {
  const int l = threadIdx.x;
  const double v = 1000.0 * (l >> 4) + (l & 15);
#pragma unroll
  for (int g = 0; g < 4; ++g) out[g * 64 + l] = static_cast<int>(bcast_group(v, g));
}

template <int V>
__global__ __launch_bounds__(64) void k_piv(double* out, long long* cyc) {
  const int l = threadIdx.x;
  v4d B, W;
  for (int r = 0; r < 4; ++r) {
    const int i = (l >> 4) + 4 * r, j = l & 15;
    B[r] = i == j ? 40.0 : 1.0 / (1.0 + i + j);
    W[r] = i == j ? 1.0 : 0.0;
  }
  bool ok = true;
  const long long t0 = clock64();
  if (V == 0) factor16_wave(B, W, l, ok);
  else factor16_chain(B, W, l, ok);
  const long long t1 = clock64();
  for (int r = 0; r < 4; ++r) out[r * 64 + l] = W[r];
  if (l == 0) cyc[0] = t1 - t0;
}

struct ProbeLds {
  double A[T * LD];
  double X[T * LD];
  double xch[2 * 4 * 256];
  ChainXch cx;
};

template <int V>
__global__ __launch_bounds__(256) void k_fact(const double* Ag, double* Xg, long long* cyc, int* okout) {
  __shared__ ProbeLds S;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  for (int e = tid; e < T * T; e += 256) S.A[(e / T) * LD + e % T] = Ag[e];
  if (tid == 0) S.cx.step = 0;
  __syncthreads();
  long long t0 = 0, t1 = 0;
  bool ok = true;
  if (V == 1) {
    v4d accA[4], accX[4];
    for (int TJ = 0; TJ < 4; ++TJ)
      for (int r = 0; r < 4; ++r) {
        const int row = ACC_ROW(w, l, r), col = ACC_COL(TJ, l);
        accA[TJ][r] = TJ >= w ? S.A[row * LD + col] : 0.0;
        accX[TJ][r] = row == col ? 1.0 : 0.0;
      }
    __syncthreads();
    t0 = clock64();
    ok = factor_tile_blk(accA, accX, w, l, S.xch);
    __syncthreads();
    t1 = clock64();
    for (int TJ = 0; TJ < 4; ++TJ)
      for (int r = 0; r < 4; ++r) S.X[ACC_ROW(w, l, r) * LD + ACC_COL(TJ, l)] = accX[TJ][r];
  } else {
    v4d a[10];
    if (w == 0) {
#pragma unroll
      for (int I = 0; I < 4; ++I)
#pragma unroll
        for (int J = I; J < 4; ++J)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            a[bidx(I, J)][r] = S.A[(16 * I + (l >> 4) + 4 * r) * LD + 16 * J + (l & 15)];
    }
    __syncthreads();
    t0 = clock64();
    if (w == 0) {
      long long st[8];
      if (V == 2) ok = factor_tile_chain<1>(a, S.cx, l, st);
      else if (V == 3) ok = factor_tile_chain<0>(a, S.cx, l, st);
      else ok = factor_tile_chain<2>(a, S.cx, l, st);
      if (l == 0 && blockIdx.x == 0)
        for (int q = 0; q < 8; ++q) cyc[16 + q] = st[q] - t0;
      // block column 3: X_33 = W_3^T
      const v4d W3 = get_blk(S.cx.W[3], l), e = ident16(l);
      v4d z = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int r = 0; r < 4; ++r) z = mfma_tn_slice(W3, e, z, r, false);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          S.X[(16 * i + (l >> 4) + 4 * r) * LD + 48 + (l & 15)] = i == 3 ? z[r] : 0.0;
    } else {
      inverse_column(S.cx, w - 1, l, S.X, LD);
    }
    __syncthreads();
    t1 = clock64();
  }
  for (int e = tid; e < T * T; e += 256) Xg[e] = S.X[(e / T) * LD + e % T];
  if (tid == 0) cyc[0] = t1 - t0;
  if (w == 0 && l == 0) okout[0] = ok;
}

int main() {
  // broadcast check
  int* dout;
  hipMalloc(&dout, 4 * 64 * 4);
  k_bcast<<<1, 64>>>(dout);
  std::vector<int> hb(256);
  hipMemcpy(hb.data(), dout, 256 * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int g = 0; g < 4; ++g)
    for (int l = 0; l < 64; ++l)
      if (hb[g * 64 + l] != 1000 * g + (l & 15)) ++bad;
  printf("bcast_group: %s (%d bad)\n", bad ? "FAIL" : "ok", bad);

  // pivot loops
  double* po; long long* pc;
  hipMalloc(&po, 256 * 8); hipMalloc(&pc, 8);
  std::vector<double> w0(256), w1(256);
  long long c0, c1;
  k_piv<0><<<1, 64>>>(po, pc); hipDeviceSynchronize();
  k_piv<0><<<1, 64>>>(po, pc); hipMemcpy(w0.data(), po, 256 * 8, hipMemcpyDeviceToHost); hipMemcpy(&c0, pc, 8, hipMemcpyDeviceToHost);
  k_piv<1><<<1, 64>>>(po, pc); hipDeviceSynchronize();
  k_piv<1><<<1, 64>>>(po, pc); hipMemcpy(w1.data(), po, 256 * 8, hipMemcpyDeviceToHost); hipMemcpy(&c1, pc, 8, hipMemcpyDeviceToHost);
  double dmax = 0, wmax = 0;
  for (int i = 0; i < 256; ++i) { dmax = std::max(dmax, std::fabs(w0[i] - w1[i])); wmax = std::max(wmax, std::fabs(w0[i])); }
  printf("factor16_wave %lld cycles, factor16_chain %lld cycles, max|dW|/max|W| = %.3e\n", c0, c1, dmax / wmax);

  std::mt19937_64 rng(5);
  std::normal_distribution<double> N(0, 1);
  std::vector<double> B(T * T), A(T * T, 0.0);
  for (auto& v : B) v = N(rng);
  for (int i = 0; i < T; ++i)
    for (int j = 0; j < T; ++j) {
      double s = 0;
      for (int k = 0; k < T; ++k) s += B[i * T + k] * B[j * T + k];
      A[i * T + j] = s + (i == j ? 1e-2 : 0.0);
    }
  std::vector<double> L(T * T, 0.0), Xr(T * T, 0.0);
  for (int j = 0; j < T; ++j) {
    double d = A[j * T + j];
    for (int k = 0; k < j; ++k) d -= L[j * T + k] * L[j * T + k];
    L[j * T + j] = std::sqrt(d);
    for (int i = j + 1; i < T; ++i) {
      double s = A[i * T + j];
      for (int k = 0; k < j; ++k) s -= L[i * T + k] * L[j * T + k];
      L[i * T + j] = s / L[j * T + j];
    }
  }
  for (int c = 0; c < T; ++c)
    for (int i = 0; i < T; ++i) {
      double s = i == c ? 1.0 : 0.0;
      for (int k = 0; k < i; ++k) s -= L[i * T + k] * Xr[k * T + c];
      Xr[i * T + c] = s / L[i * T + i];
    }
  double *dA, *dX; long long* cyc; int* ok;
  hipMalloc(&dA, T * T * 8); hipMalloc(&dX, T * T * 8); hipMalloc(&cyc, 8 * 1024); hipMalloc(&ok, 4);
  hipMemcpy(dA, A.data(), T * T * 8, hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int V = 1; V < 5; ++V) {
    auto launch = [&](int n) {
      if (V == 1) k_fact<1><<<n, 256>>>(dA, dX, cyc, ok);
      else if (V == 2) k_fact<2><<<n, 256>>>(dA, dX, cyc, ok);
      else if (V == 3) k_fact<3><<<n, 256>>>(dA, dX, cyc, ok);
      else k_fact<4><<<n, 256>>>(dA, dX, cyc, ok);
    };
    launch(1);
    hipDeviceSynchronize();
    launch(1);
    hipDeviceSynchronize();
    std::vector<double> X(T * T); int okh; long long c;
    hipMemcpy(X.data(), dX, T * T * 8, hipMemcpyDeviceToHost);
    hipMemcpy(&okh, ok, 4, hipMemcpyDeviceToHost);
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    double err = 0, mx = 0;
    for (int i = 0; i < T * T; ++i) { err = std::max(err, std::fabs(X[i] - Xr[i])); mx = std::max(mx, std::fabs(Xr[i])); }
    hipEventRecord(e0);
    for (int it = 0; it < 200; ++it) launch(1);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("%s: ok=%d  max|X-Xref|/max|Xref| = %.3e  clock64 ticks = %lld  launch = %.2f us\n",
           V == 1 ? "factor_tile_blk  " : (V == 2 ? "chain (hooks)    " : (V == 3 ? "chain (no hooks) " : "chain (no deferred, wrong)")), okh, err / mx, c,
           ms * 1e3 / 200);
    if (V > 1) {
      long long st[8];
      hipMemcpy(st, cyc + 16, 64, hipMemcpyDeviceToHost);
      printf("   step stamps (factor16 done / published):");
      for (int q = 0; q < 8; ++q) printf(" %lld", st[q]);
      printf("\n");
    }
  }
  return 0;
}
