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

#include <type_traits>

#include "kernels.hpp"
#include "f16wave.h"

namespace dynohip {

namespace {

constexpr int T = kTile;
constexpr int LD = T + 4;            // padded LDS row stride (doubles)


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
// The k order of the 64-deep LDS-operand products: in k-block K (16 wide)
// the s-th MFMA of lane group lk = l >> 4 takes k = 16K + 4 lk + s, so a
// lane's four operands of a k-block are contiguous and come in two 16-byte
// reads (ds_read_b128) instead of four 8-byte ones; both operands of a
// product use the same order. (tools/pivot_probe: 98 instead of 123 cycles
// per f64 MFMA fed from LDS.)
typedef double d2v __attribute__((ext_vector_type(2)));
struct Kq {
  d2v lo, hi;
  __device__ __forceinline__ double operator[](int s) const { return s < 2 ? lo[s] : hi[s - 2]; }
};
__device__ __forceinline__ Kq ld_kq(const double* row, int K, int lk) {
  const d2v* p = reinterpret_cast<const d2v*>(row + 16 * K + 4 * lk);
  return Kq{p[0], p[1]};
}

__device__ __forceinline__ void mfma_abt_acc(const double* As, const double* Bs, int wave, int lane, v4d acc[2][2]) {
  const int i0 = 32 * (wave >> 1), j0 = 32 * (wave & 1);
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int K = 0; K < 4; ++K) {
    const Kq a0 = ld_kq(As + (i0 + li) * LD, K, lk), a1 = ld_kq(As + (i0 + 16 + li) * LD, K, lk);
    const Kq b0 = ld_kq(Bs + (j0 + li) * LD, K, lk), b1 = ld_kq(Bs + (j0 + 16 + li) * LD, K, lk);
    // (each accumulator's four k-steps back to back: consecutive f64 MFMAs
    // on one accumulator issue faster than rotating over four)
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0[s4], b0[s4], acc[0][0], 0, 0, 0);
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0[s4], b1[s4], acc[0][1], 0, 0, 0);
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[s4], b0[s4], acc[1][0], 0, 0, 0);
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[s4], b1[s4], acc[1][1], 0, 0, 0);
  }
}

// element (row, col) of the quadrant result held by this lane
#define MFMA_ROW(wave, lane, ti, r) (32 * ((wave) >> 1) + 16 * (ti) + ((lane) >> 4) + 4 * (r))
#define MFMA_COL(wave, lane, tj) (32 * ((wave) & 1) + 16 * (tj) + ((lane) & 15))

#ifdef DYNOHIP_TASK_CLOCK
// per-task timestamps of the last k_factor_persist launch (s_memrealtime,
// 100 MHz): dequeue, dependencies met, factor start, factor end, done; and
// the worker; sub-phases and the factorisation's block steps (tools/task_clock.py)
__device__ unsigned long long g_tclk[32][32768];
#define TCLK(idx, q, v) \
  do {                  \
    if (threadIdx.x == 0 && (q) < 32768) g_tclk[idx][q] = (v); \
  } while (0)
// lane 0 of the calling wave (s_memtime: shader clock cycles)
#define TCLKW(idx, q) \
  do {                  \
    if ((threadIdx.x & 63) == 0 && (q) < 32768) g_tclk[idx][q] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define TCLKW(idx, q) \
  do {                  \
  } while (0)
#define TCLK(idx, q, v) \
  do {                  \
  } while (0)
#endif
#ifdef DYNOHIP_TASK_CLOCK
__device__ __forceinline__ unsigned long long rtc() { return __builtin_amdgcn_s_memrealtime(); }
#endif

__device__ __forceinline__ double* slot_ptr(const TileDev& b, int32_t slot) {
  return b.slots + static_cast<int64_t>(slot) * T * T;
}

// MFMA accumulator layout of a 64x64 tile over 4 waves: wave w holds the 16
// rows 16w.. as four 16x16 tiles TJ; lane l, reg r of tile TJ is element
// (16w + (l>>4) + 4r, 16TJ + (l&15)).
#define ACC_ROW(w, l, r) (16 * (w) + ((l) >> 4) + 4 * (r))
#define ACC_COL(TJ, l) (16 * (TJ) + ((l) & 15))

// acc (+)= Y^T Z for 16x16 blocks Y, Z in accumulator layout (K = 16)
__device__ __forceinline__ v4d mfma_tn(const v4d& Y, const v4d& Z, v4d acc, bool neg) {
#pragma unroll
  for (int r = 0; r < 4; ++r) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(neg ? -Y[r] : Y[r], Z[r], acc, 0, 0, 0);
  return acc;
}

// Factor the 64x64 tile held as upper 16x16 blocks (wave w: accA[TJ] =
// block (w, TJ), TJ >= w, full symmetric input) and build L^-1 in accX
// (wave w: block row w; starts as I). Four block steps KB, one barrier each:
//   wave KB:   U_KK and W = U_KK^-1 in-wave; U row KB = W^T A[KB][TJ]
//              (TJ > KB), published;
//   wave KB-1: finishes row KB-1 of the inverse, Xf = W_{KB-1}^T X[KB-1][TJ]
//              (TJ <= KB-1), published in the slots the U row leaves free;
//   waves v > KB, after the barrier: A[v][TJ] -= U[KB][v]^T U[KB][TJ] (TJ >= v),
//              and the inverse rows lagging one step,
//              X[v][TJ] -= U[KB-1][v]^T Xf[KB-1][TJ] (TJ <= KB-1).
// The inverse work thus runs on waves that would otherwise wait, and only
// the last inverse row follows the final barrier. Each wave keeps its
// previous U block and its own W in registers.
// xch: 2 x 4 blocks x 256 doubles of LDS; dscr: 16 doubles per wave.
// idle(KB) runs at the top of block step KB on every wave but the factoring
// one (wave KB): the caller spreads its independent MFMA work (pending
// updates) over the periods in which a wave would otherwise wait.
struct NoHook {
  __device__ void operator()(int) const {}
};

template <int w, class Idle = NoHook>
__device__ bool factor_tile_blk_w(v4d (&accA)[4], v4d (&accX)[4], int l, double* xch, double* dscr, Idle&& idle,
                                  int q) {
  bool ok = true;
  v4d Wmine = v4d{0.0, 0.0, 0.0, 0.0};   // W of this wave's diagonal block
  v4d Uprev = v4d{0.0, 0.0, 0.0, 0.0};   // U[KB-1][w]
  v4d Udefer = v4d{0.0, 0.0, 0.0, 0.0};  // U[KB-2][w] of the deferred inverse update
  // the inverse update of the wave that factors next is deferred past its
  // own factorisation; xch slots < KB-1 of the previous buffer stay intact
  // for it (nobody else writes them before it reads)
  auto x_update = [&](const v4d& U, const double* buf, int nblk) {
#pragma unroll
    for (int TJ = 0; TJ < 4; ++TJ)
      if (TJ < nblk) {
        v4d Z;
#pragma unroll
        for (int r = 0; r < 4; ++r) Z[r] = buf[TJ * 256 + r * 64 + l];
        accX[TJ] = mfma_tn(U, Z, accX[TJ], true);
      }
  };
#pragma unroll
  for (int KB = 0; KB < 4; ++KB) {
    double* xb = xch + (KB & 1) * 4 * 256;
    double* xp = xch + ((KB + 1) & 1) * 4 * 256;  // previous step's buffer
    if (w != KB) idle(KB);
    if (w == KB) {
#pragma unroll
      for (int r = 0; r < 4; ++r) Wmine[r] = ((l >> 4) + 4 * r == (l & 15)) ? 1.0 : 0.0;
      TCLKW(16 + 4 * KB, q);
      factor16(accA[KB], Wmine, l, ok, dscr);
      TCLKW(17 + 4 * KB, q);
#pragma unroll
      for (int TJ = KB + 1; TJ < 4; ++TJ) {
        v4d z = v4d{0.0, 0.0, 0.0, 0.0};
        accA[TJ] = mfma_tn(Wmine, accA[TJ], z, false);
#pragma unroll
        for (int r = 0; r < 4; ++r) xb[TJ * 256 + r * 64 + l] = accA[TJ][r];
      }
    }
    if (w == KB) TCLKW(18 + 4 * KB, q);
    if (KB >= 1 && w == KB - 1) {
      // final inverse row KB-1 (all its updates from rows < KB-1 applied)
#pragma unroll
      for (int TJ = 0; TJ < KB; ++TJ) {
        v4d z = v4d{0.0, 0.0, 0.0, 0.0};
        accX[TJ] = mfma_tn(Wmine, accX[TJ], z, false);
#pragma unroll
        for (int r = 0; r < 4; ++r) xb[TJ * 256 + r * 64 + l] = accX[TJ][r];
      }
    }
    __syncthreads();
    TCLK(12 + KB, q, rtc());
    if (w == KB) TCLKW(19 + 4 * KB, q);
    if (w > KB) {
      v4d Uv;
#pragma unroll
      for (int r = 0; r < 4; ++r) Uv[r] = xb[w * 256 + r * 64 + l];
#pragma unroll
      for (int TJ = 0; TJ < 4; ++TJ) {
        if (TJ < w) continue;
        v4d Z;
#pragma unroll
        for (int r = 0; r < 4; ++r) Z[r] = xb[TJ * 256 + r * 64 + l];
        accA[TJ] = mfma_tn(Uv, Z, accA[TJ], true);
      }
      if (w == KB + 1) {
        Udefer = Uprev;            // Xf[KB-1] (slots < KB of xb) applied after my factorisation
      } else if (KB >= 1) {
        x_update(Uprev, xb, KB);   // Xf[KB-1]
      }
      Uprev = Uv;
    } else if (w == KB) {
      // after my factorisation: the deferred Xf[KB-2] (previous buffer),
      // then Xf[KB-1]
      if (KB >= 2) x_update(Udefer, xp, KB - 1);
      if (KB >= 1) x_update(Uprev, xb, KB);
    }
  }
  if (w == 3) {
    // last inverse row
#pragma unroll
    for (int TJ = 0; TJ < 4; ++TJ) {
      v4d z = v4d{0.0, 0.0, 0.0, 0.0};
      accX[TJ] = mfma_tn(Wmine, accX[TJ], z, false);
    }
  }
  return ok;
}

// The wave index is a template parameter of the body above: with a runtime
// index the compiler merges the four "if (w == KB)" branches into one and
// addresses accA by w through 16-way select chains.
template <class Idle = NoHook>
__device__ __forceinline__ bool factor_tile_blk(v4d (&accA)[4], v4d (&accX)[4], int w, int l, double* xch,
                                                double* dscr, Idle&& idle = Idle(), int q = 0) {
  switch (__builtin_amdgcn_readfirstlane(w)) {
    case 0: return factor_tile_blk_w<0>(accA, accX, l, xch, dscr, idle, q);
    case 1: return factor_tile_blk_w<1>(accA, accX, l, xch, dscr, idle, q);
    case 2: return factor_tile_blk_w<2>(accA, accX, l, xch, dscr, idle, q);
    default: return factor_tile_blk_w<3>(accA, accX, l, xch, dscr, idle, q);
  }
}


// ---- global memory access of the factorisation --------------------------
// The level kernels (SC1 = false) read tiles written by earlier launches
// with plain loads. The one-launch dataflow kernel (SC1 = true) hands tiles
// between workgroups inside the launch, following cdna_hip_programming.md
// Guideline 16 R1: every tile element, contribution and pending operand
// written in the launch is stored write-through (sc1) and drained before the
// slot's write counter is bumped, and every load of such data is an sc1 load
// (16-byte buffer loads for whole tiles, 8-byte atomic loads otherwise), so
// no acquire fence is needed.

template <bool SC1>
__device__ __forceinline__ double gld(const double* p) {
  if constexpr (SC1) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}
template <bool SC1>
__device__ __forceinline__ void gst(double* p, double v) {
  if constexpr (SC1) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

// a tile base pointer is wave-uniform; make that visible to the compiler so
// the buffer descriptor lives in SGPRs
__device__ __forceinline__ const double* uniform_ptr(const double* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
  return reinterpret_cast<const double*>((static_cast<uint64_t>(hi) << 32) | lo);
}

template <bool SC1>
__device__ __forceinline__ void load_tile_lds_t(const double* __restrict__ src, double* dst, int tid) {
  if constexpr (SC1) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(uniform_ptr(src)), 0, T * T * 8, 0x00020000);
    d2v v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
      v[i] = __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(rs, (tid + 256 * i) * 16, 0, 16));
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = tid + 256 * i, rr = (2 * e) / T, cc = (2 * e) % T;
      dst[rr * LD + cc] = v[i].x;
      dst[rr * LD + cc + 1] = v[i].y;
    }
  } else {
    load_tile_lds(src, dst, tid, 256);
  }
}

// Issue the loads of up to four 64x64 tiles into LDS before any of the
// stores, so their latencies overlap (one round trip instead of four). A
// null source skips its tile. (Fixed operand positions, no pointer arrays:
// those would go through scratch and turn the LDS stores into flat stores.)
template <bool SC1>
__device__ __forceinline__ void load_tiles_lds(const double* s0, double* d0, const double* s1, double* d1,
                                               const double* s2, double* d2, const double* s3, double* d3,
                                               int tid) {
  const double* const src[4] = {s0, s1, s2, s3};
  d2v v[4][8];
#pragma unroll
  for (int t = 0; t < 4; ++t)
    if (src[t]) {
      if constexpr (SC1) {
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(uniform_ptr(src[t])), 0, T * T * 8, 0x00020000);
#pragma unroll
        for (int i = 0; i < 8; ++i)
          v[t][i] = __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(rs, (tid + 256 * i) * 16, 0, 16));
      } else {
        const d2v* s2v = reinterpret_cast<const d2v*>(src[t]);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[t][i] = s2v[tid + 256 * i];
      }
    }
  auto put = [&](int t, double* d) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = tid + 256 * i, rr = (2 * e) / T, cc = (2 * e) % T;
      d[rr * LD + cc] = v[t][i].x;
      d[rr * LD + cc + 1] = v[t][i].y;
    }
  };
  if (s0) put(0, d0);
  if (s1) put(1, d1);
  if (s2) put(2, d2);
  if (s3) put(3, d3);
}

// a 64x64 tile into registers (16 bytes per load, 8 per thread) and from
// them into LDS (row stride LD)
template <bool SC1>
__device__ __forceinline__ void tile_regs(const double* __restrict__ src, d2v (&v)[8], int tid) {
  if constexpr (SC1) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(uniform_ptr(src)), 0, T * T * 8, 0x00020000);
#pragma unroll
    for (int i = 0; i < 8; ++i)
      v[i] = __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(rs, (tid + 256 * i) * 16, 0, 16));
  } else {
    const d2v* s2v = reinterpret_cast<const d2v*>(src);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = s2v[tid + 256 * i];
  }
}
__device__ __forceinline__ void regs_tile(const d2v (&v)[8], double* d, int tid) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int e = tid + 256 * i, rr = (2 * e) / T, cc = (2 * e) % T;
    d[rr * LD + cc] = v[i].x;
    d[rr * LD + cc + 1] = v[i].y;
  }
}

// dst -= sum over the task's pairs of A B^T: the destination and the first
// pair's operands are fetched in one round trip; each further pair's while
// the previous pair's MFMAs run
struct NoWait {
  __device__ void operator()() const {}
};

template <bool SC1, class LateWait = NoWait>
// pa0 / pb0: the first pair's slots when the caller fetched them before the
// dependency wait (-1: read them here). late(): called between the
// destination loads and the operand loads (the dataflow kernel waits there
// for the operand tiles, whose producers usually finish last)
__device__ __forceinline__ void run_update(const TileDev& b, const TileTask& tk, const int32_t* __restrict__ pairs,
                                           double* Qs, double* Rs, int tid, int w, int l, int32_t pa0 = -1,
                                           int32_t pb0 = -1, LateWait&& late = LateWait()) {
  double* dst = slot_ptr(b, tk.dst);
  double old[2][2][4];
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < 2; ++tj)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) old[ti][tj][rr] = gld<SC1>(dst + MFMA_ROW(w, l, ti, rr) * T + MFMA_COL(w, l, tj));
  late();
  v4d acc[2][2];
  zero_acc(acc);
  if (tk.po_end > tk.po_beg) {
    const int32_t pa = pa0 >= 0 ? pa0 : pairs[2 * tk.po_beg], pb = pa0 >= 0 ? pb0 : pairs[2 * tk.po_beg + 1];
    load_tiles_lds<SC1>(slot_ptr(b, pa), Qs, pb != pa ? slot_ptr(b, pb) : nullptr, Rs, nullptr, nullptr, nullptr,
                        nullptr, tid);
    __syncthreads();
  }
  // pair e is in LDS; pair e + 1's tiles are loaded into registers while
  // pair e's MFMAs run (grouped updates carry ~2 pairs: one round trip less)
  for (int e = tk.po_beg; e < tk.po_end; ++e) {
    const int32_t pa = e == tk.po_beg && pa0 >= 0 ? pa0 : pairs[2 * e];
    const int32_t pb = e == tk.po_beg && pa0 >= 0 ? pb0 : pairs[2 * e + 1];
    const bool more = e + 1 < tk.po_end;
    d2v nv[2][8];
    int32_t na = -1, nb = -1;
    if (more) {
      na = pairs[2 * (e + 1)];
      nb = pairs[2 * (e + 1) + 1];
      tile_regs<SC1>(slot_ptr(b, na), nv[0], tid);
      if (nb != na) tile_regs<SC1>(slot_ptr(b, nb), nv[1], tid);
    }
    mfma_abt_acc(Qs, pb != pa ? Rs : Qs, w, l, acc);
    if (more) {
      __syncthreads();
      regs_tile(nv[0], Qs, tid);
      if (nb != na) regs_tile(nv[1], Rs, tid);
      __syncthreads();
    }
  }
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < 2; ++tj)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        gst<SC1>(dst + MFMA_ROW(w, l, ti, rr) * T + MFMA_COL(w, l, tj), old[ti][tj][rr] - acc[ti][tj][rr]);
}

// A_kk -= L(k,c) L(k,c)^T on this wave's upper blocks (w, TJ >= w), K = 64
__device__ __forceinline__ void diag_pending(v4d (&accA)[4], const double* Ps, int w, int l) {
  const int li = l & 15, lk = l >> 4;
#pragma unroll
  for (int K = 0; K < 4; ++K) {
    const Kq a = ld_kq(Ps + (16 * w + li) * LD, K, lk);
#pragma unroll
    for (int TJ = 0; TJ < 4; ++TJ)
      if (TJ >= w) {
        const Kq bq = ld_kq(Ps + (16 * TJ + li) * LD, K, lk);
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
          accA[TJ] = __builtin_amdgcn_mfma_f64_16x16x4f64(-a[s4], bq[s4], accA[TJ], 0, 0, 0);
      }
  }
}



struct TaskLds {
  double Ps[T * LD];   // pending diagonal operand L(k, c) -> later L_kk^-1; second pair operand otherwise
  double Qs[T * LD];   // pair operand A
  double As[T * LD];   // own tile (i, k)
  double Xch[2 * 4 * 256];
  double Ust[16 * 256];  // own panels: W_c = U_cc^-1 at [c][c], U[c][TJ] at [c][TJ] (16x16, accumulator layout)
  double rpart[4][T];
  double vv[T];        // r_k minus the contributions of eliminated columns
  double yv[T];        // y_k = L_kk^-1 vv
  double tv[4][16];    // forward substitution scratch, per block
  // own panels: per block step KB, "U row KB published" flags holding the
  // task's sequence number (flagA: W_KB and U[KB][KB+1], flagB: the whole
  // row), and "y_KB out" (factor_own_w)
  int flagA[4], flagB[4], yflag[4];
};

// Hand-offs between the waves of one workgroup through LDS: the producer
// drains its LDS writes (lgkmcnt(0)) and then stores the flag; a consumer
// polls the flag and only then issues its loads (LDS operations of one wave
// complete in order, so a consumer that sees the flag sees the data).
__device__ __forceinline__ void lds_flag_set(int* f, int v) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if ((threadIdx.x & 63) == 0) __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  asm volatile("" ::: "memory");
}
// The poll is one opaque loop of five instructions (the compiler would
// otherwise duplicate the code around every inlined spin loop).
__device__ __forceinline__ void lds_flag_wait(const int* f, int v) {
  const unsigned a = static_cast<unsigned>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const int*)f));
  const int vs = __builtin_amdgcn_readfirstlane(v);   // (wave-uniform; an SGPR operand)
  int t;
  int st;
  asm volatile(
      "1:\n\t"
      "ds_read_b32 %0, %2\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "v_readfirstlane_b32 %1, %0\n\t"
      "s_cmp_lg_u32 %1, %3\n\t"
      "s_cbranch_scc1 1b"
      : "=&v"(t), "=&s"(st)
      : "v"(a), "s"(vs)
      : "memory", "scc");
}

// Launch-invariant inputs of a panel task: operand slots, the entries of
// tile row k and r_k. They are fetched before the dependency wait, so that
// after it a single round trip brings every operand.
constexpr int kCsMax = 8;   // contribution entries per wave in that round trip
struct PanelPre {
  int32_t pd, qa, rb;       // fast path: pending diagonal operand, own pending pair (-1: none)
  int32_t rbeg, rend;       // entries of tile row k
  int32_t cs[kCsMax];       // this wave's contribution slots, entries rbeg + w + 4j (-1: none)
  double rk;                // r_k[lane]
  bool fast;                // at most one pending pair each
};

__device__ __forceinline__ PanelPre panel_prefetch(const TileDev& b, const TileTask& tk,
                                                   const int32_t* __restrict__ pairs, const double* __restrict__ r,
                                                   int w, int l) {
  PanelPre p;
  const bool own = tk.i != tk.k;
  const int npd = tk.pd_end - tk.pd_beg, npo = own ? tk.po_end - tk.po_beg : 0;
  p.pd = npd == 1 ? pairs[2 * tk.pd_beg] : -1;
  p.qa = npo == 1 ? pairs[2 * tk.po_beg] : -1;
  p.rb = npo == 1 ? pairs[2 * tk.po_beg + 1] : -1;
  // the own pair's second operand L(k,c) must be the first one or the pending
  // diagonal operand already in Ps (always so in practice); else the slow path
  p.fast = npd <= 1 && npo <= 1 && (p.rb == p.qa || p.rb == p.pd);
  p.rbeg = b.row_start[tk.k];
  p.rend = b.row_start[tk.k + 1];
  const int wu = __builtin_amdgcn_readfirstlane(w);
#pragma unroll
  for (int j = 0; j < kCsMax; ++j) {
    const int e = p.rbeg + wu + 4 * j;
    p.cs[j] = (e < p.rend && b.row_col[e] != tk.k) ? b.row_slot[e] : -1;
  }
  p.rk = r[static_cast<int64_t>(tk.k) * T + l];
  return p;
}

// acc += -P_bi P_bj^T for 16x16 blocks (bi, bj) of a 64x64 LDS operand P,
// in accumulator layout (the pending update of diagonal block (bi, bj)).
__device__ __forceinline__ v4d pend_block(v4d acc, const double* Ps, int bi, int bj, int l) {
  const int li = l & 15, lk = l >> 4;
  // one accumulator chain (tools/pivot_probe: 86 cycles per LDS-fed f64
  // MFMA against 99 rotating over four)
  v4d c = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int K = 0; K < 4; ++K) {
    const Kq a = ld_kq(Ps + (16 * bi + li) * LD, K, lk), bq = ld_kq(Ps + (16 * bj + li) * LD, K, lk);
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) c = __builtin_amdgcn_mfma_f64_16x16x4f64(-a[s4], bq[s4], c, 0, 0, 0);
  }
  return acc + c;
}

// sum over the 16 lanes of a row group (lanes with equal l >> 4), with DPP
// moves only: quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror
// (a symmetric tree: every lane gets the same, bit-identical sum)
__device__ __forceinline__ double sum16(double v) {
  v += __builtin_amdgcn_update_dpp(__builtin_nan(""), v, 0xB1, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(__builtin_nan(""), v, 0x4E, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(__builtin_nan(""), v, 0x141, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(__builtin_nan(""), v, 0x140, 0xf, 0xf, true);
  return v;
}

// ---- own panels (i != k): the factorisation with the TRSM folded in ----
// L(i,k) = A(i,k) U^-1 (U = L_kk^T) by block forward substitution over the
// four 16-column blocks c, interleaved with the block steps of the diagonal
// factorisation: wave w keeps XT[c] = (block (w, c) of L(i,k))^T and forms
//   XT[c] = W_c^T (A(w,c)^T - sum_{c' < c} U[c'][c]^T XT[c'])
// as soon as W_c = U_cc^-1 and U[c'][c] are out (the U blocks stay in LDS,
// Ust). y_k = L_kk^-1 vv is the same substitution on the right-hand side,
// done by the factoring wave of each step. No explicit L_kk^-1 is formed
// (the diagonal task stores it for the backward substitution), so there is
// no inverse row to finish after the last step: one substitution block per
// wave follows the final barrier instead of the whole TRSM.
//
// The own-tile pending update A(i,k) -= Q R^T runs in four column chunks
// (16 MFMAs each, into As) and the substitution blocks are scheduled per wave
// into the slots of the factorisation in which the wave would otherwise
// wait: I<KB> before block step KB (not on the factoring wave), B<KB> after
// its barrier. A chunk precedes the substitution block of its columns; the
// wave that factors next does nothing extra after the barrier before its
// step. y_c = W_c^T (vv_c - sum_{c' < c} U[c'][c]^T y_c') is latency-bound
// small work: it runs after barrier c (its inputs are out by then), off the
// factoring wave's path. Actions: 0x10 + c = chunk c, 0x20 + c = substitution
// block c, 0x30 + c = y_c.
constexpr int kOwnAct[4][8][4] = {
    // I0           B0                          I1                  B1                          I2            B2                     I3            B3
    {{0, 0, 0, 0}, {0x30, 0x10, 0x20, 0x11}, {0, 0, 0, 0}, {0x31, 0x21, 0x12, 0}, {0, 0, 0, 0}, {0x32, 0x22, 0x13, 0}, {0, 0, 0, 0}, {0x23, 0, 0, 0}},
    {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0x10, 0x20, 0x11, 0x21}, {0, 0, 0, 0}, {0x12, 0x22, 0x13, 0}, {0, 0, 0, 0}, {0x33, 0x23, 0, 0}},
    {{0x10, 0, 0, 0}, {0x20, 0, 0, 0}, {0x11, 0x12, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0x21, 0x22, 0, 0}, {0x13, 0, 0, 0}, {0x23, 0, 0, 0}},
    {{0x10, 0x11, 0, 0}, {0x20, 0, 0, 0}, {0x12, 0x13, 0, 0}, {0x21, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0x22, 0x23, 0, 0}},
};

__device__ __forceinline__ v4d ld_blk(const double* p, int l) {
  v4d v;
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = p[r * 64 + l];
  return v;
}
__device__ __forceinline__ void st_blk(double* p, const v4d& v, int l) {
#pragma unroll
  for (int r = 0; r < 4; ++r) p[r * 64 + l] = v[r];
}

// sum over the four row groups (lanes l, l^16, l^32, l^48)
__device__ __forceinline__ double sum_groups(double v) {
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return v;
}

template <int w, class DiagPend, class Chunk>
__device__ bool factor_own_w(v4d (&accA)[4], v4d (&XT)[4], int l, TaskLds& S, DiagPend&& diagpend, Chunk&& chunk,
                             int q, int seq) {
  bool ok = true;
  const int li = l & 15, g = l >> 4;
  double* const U = S.Ust;
  auto Ublk = [&](int c, int tj) { return U + (c * 4 + tj) * 256; };
  auto subst = [&](int c) {
    lds_flag_wait(&S.flagB[c], seq);   // W_c and every U[c'][c], c' < c
    v4d Tm;   // A(w, c)^T: element (j = g + 4r, i = li) = A[16w + i][16c + j]
#pragma unroll
    for (int r = 0; r < 4; ++r) Tm[r] = S.As[(16 * w + li) * LD + 16 * c + g + 4 * r];
    // the c' terms as independent chains, subtracted in order
    v4d sum[3];
#pragma unroll
    for (int cp = 0; cp < 3; ++cp)
      if (cp < c) sum[cp] = mfma_tn(ld_blk(Ublk(cp, c), l), XT[cp], v4d{0.0, 0.0, 0.0, 0.0}, false);
#pragma unroll
    for (int cp = 0; cp < 3; ++cp)
      if (cp < c) Tm -= sum[cp];
    XT[c] = mfma_tn(ld_blk(Ublk(c, c), l), Tm, v4d{0.0, 0.0, 0.0, 0.0}, false);
  };
  auto ystep = [&](int c) {   // y_c = W_c^T (vv_c - sum_{c' < c} U[c'][c]^T y_c')
    lds_flag_wait(&S.flagB[c], seq);
    if (c > 0) lds_flag_wait(&S.yflag[c - 1], seq);
    double part = 0.0;
#pragma unroll
    for (int cp = 0; cp < 3; ++cp)
      if (cp < c) {
        const v4d u = ld_blk(Ublk(cp, c), l);
#pragma unroll
        for (int r = 0; r < 4; ++r) part += u[r] * S.yv[16 * cp + g + 4 * r];
      }
    const double t = S.vv[16 * c + li] - sum_groups(part);
    if (g == 0) S.tv[c][li] = t;
    const v4d Wc = ld_blk(Ublk(c, c), l);
    double yp = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r) yp += Wc[r] * S.tv[c][g + 4 * r];
    yp = sum_groups(yp);
    if (g == 0) S.yv[16 * c + li] = yp;
    lds_flag_set(&S.yflag[c], seq);
  };
  auto act = [&](int slot) {
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int x = kOwnAct[w][slot][a];
      if (x >= 0x30) ystep(x - 0x30);
      else if (x >= 0x20) subst(x - 0x20);
      else if (x >= 0x10) chunk(x - 0x10);
    }
  };
  // step KB's trailing update of this wave's blocks TJ in [t0, t1)
  auto trailing = [&](int KB, int t0, int t1) {
    const v4d Uv = ld_blk(Ublk(KB, w), l);
#pragma unroll
    for (int TJ = 0; TJ < 4; ++TJ)
      if (TJ >= t0 && TJ < t1) accA[TJ] = mfma_tn(Uv, ld_blk(Ublk(KB, TJ), l), accA[TJ], true);
  };
  // No barrier per block step: the waves hand the U rows over through LDS
  // flags, so a wave waits only for the data it reads, not for the other
  // waves' chunk and substitution work. The wave that factors next takes
  // step KB's update of its diagonal block as soon as W_KB and U[KB][KB+1]
  // are out (flagA), factors, and only then applies step KB's update to its
  // other blocks (flagB): each block still receives its updates in step order.
#pragma unroll
  for (int KB = 0; KB < 4; ++KB) {
    if (w != KB) {
      if (KB == 0) diagpend();
      act(2 * KB);
    } else {
      v4d Wm;
#pragma unroll
      for (int r = 0; r < 4; ++r) Wm[r] = (g + 4 * r == li) ? 1.0 : 0.0;
      TCLKW(16 + 4 * KB, q);
      factor16(accA[KB], Wm, l, ok, &S.rpart[w][0]);
      TCLKW(17 + 4 * KB, q);
      if (KB >= 1 && KB + 1 < 4) {
        // the rest of step KB-1's update of this wave's blocks, off the
        // diagonal block's path but before this row's U blocks use them
        lds_flag_wait(&S.flagB[KB - 1], seq);
        trailing(KB - 1, KB + 1, 4);
      }
      st_blk(Ublk(KB, KB), Wm, l);
      if (KB + 1 < 4) {
        accA[KB + 1] = mfma_tn(Wm, accA[KB + 1], v4d{0.0, 0.0, 0.0, 0.0}, false);
        st_blk(Ublk(KB, KB + 1), accA[KB + 1], l);
      }
      lds_flag_set(&S.flagA[KB], seq);
#pragma unroll
      for (int TJ = KB + 2; TJ < 4; ++TJ) {
        accA[TJ] = mfma_tn(Wm, accA[TJ], v4d{0.0, 0.0, 0.0, 0.0}, false);
        st_blk(Ublk(KB, TJ), accA[TJ], l);
      }
      lds_flag_set(&S.flagB[KB], seq);
      TCLKW(18 + 4 * KB, q);
    }
    if (w == KB) TCLKW(19 + 4 * KB, q);
    if (w == KB + 1) {
      lds_flag_wait(&S.flagA[KB], seq);
      trailing(KB, w, w + 1);   // the next diagonal block: the critical path
    } else if (w > KB + 1) {
      lds_flag_wait(&S.flagB[KB], seq);
      trailing(KB, w, 4);
    }
    act(2 * KB + 1);
  }
  return ok;
}

template <class DiagPend, class Chunk>
__device__ __forceinline__ bool factor_own(v4d (&accA)[4], v4d (&XT)[4], int w, int l, TaskLds& S,
                                           DiagPend&& diagpend, Chunk&& chunk, int q, int seq) {
  switch (__builtin_amdgcn_readfirstlane(w)) {
    case 0: return factor_own_w<0>(accA, XT, l, S, diagpend, chunk, q, seq);
    case 1: return factor_own_w<1>(accA, XT, l, S, diagpend, chunk, q, seq);
    case 2: return factor_own_w<2>(accA, XT, l, S, diagpend, chunk, q, seq);
    default: return factor_own_w<3>(accA, XT, l, S, diagpend, chunk, q, seq);
  }
}

template <bool SC1, class LateWait = NoWait>
__device__ __forceinline__ void panel_task(const TileDev& b, const TileTask& tk, const int32_t* __restrict__ pairs,
                                           const PanelPre& p, double* __restrict__ Linv, double* __restrict__ contrib,
                                           double* __restrict__ y, int* fail, TaskLds& S, int q = 0,
                                           LateWait&& late = LateWait(), int seq = 1) {
  double* const Ps = S.Ps;
  double* const Qs = S.Qs;
  double* const As = S.As;
  const int tid = threadIdx.x;
  const int w = tid >> 6, l = tid & 63;
  const int li = l & 15, lk = l >> 4;
  const bool own = tk.i != tk.k;
  // (1) two round trips: first what the dependency-ready tiles hold (the
  // diagonal tile, stored symmetric, into registers, and the own tile into
  // LDS), issued before the wait for the pending operands (late(): in the
  // dataflow kernel the tiles the previous task on the critical path just
  // produced), then those operand tiles into LDS and the right-hand side
  // contributions L(k,c) y_c of eliminated columns
  v4d accA[4];
  const double* diag = slot_ptr(b, tk.diag);
#pragma unroll
  for (int TJ = 0; TJ < 4; ++TJ)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = ACC_ROW(w, l, rr), col = ACC_COL(TJ, l);
      accA[TJ][rr] = TJ >= w ? gld<SC1>(diag + row * T + col) : 0.0;
    }
  if (p.fast && own)
    load_tiles_lds<SC1>(nullptr, Ps, slot_ptr(b, tk.dst), As, nullptr, Qs, nullptr, nullptr, tid);
  late();
  double cv[kCsMax];
#pragma unroll
  for (int j = 0; j < kCsMax; ++j)
    cv[j] = p.cs[j] >= 0 ? gld<SC1>(contrib + static_cast<int64_t>(p.cs[j]) * T + l) : 0.0;
  if (p.fast) {
    load_tiles_lds<SC1>(p.pd >= 0 ? slot_ptr(b, p.pd) : nullptr, Ps, nullptr, As,
                        p.qa >= 0 ? slot_ptr(b, p.qa) : nullptr, Qs, nullptr, nullptr, tid);
  }
  {
    double sacc = 0.0;
#pragma unroll
    for (int j = 0; j < kCsMax; ++j)
      if (p.cs[j] >= 0) sacc += cv[j];
    for (int e = p.rbeg + w + 4 * kCsMax; e < p.rend; e += 4)   // long rows (rare)
      if (b.row_col[e] != tk.k) sacc += gld<SC1>(contrib + static_cast<int64_t>(b.row_slot[e]) * T + l);
    S.rpart[w][l] = sacc;
  }
  TCLK(6, q, rtc());
  if (!p.fast) {
    // several pending pairs (the first column of a separator, fed by two
    // subtrees at once): applied before the factor, the own tile and the
    // first own pair fetched in one round trip, and each further operand
    // tile fetched into registers while the previous one's MFMAs run
    if (own) {
      const bool hp = tk.po_end > tk.po_beg;
      const int32_t pa0 = hp ? pairs[2 * tk.po_beg] : -1, pb0 = hp ? pairs[2 * tk.po_beg + 1] : -1;
      load_tiles_lds<SC1>(slot_ptr(b, tk.dst), As, hp ? slot_ptr(b, pa0) : nullptr, Qs,
                          hp && pb0 != pa0 ? slot_ptr(b, pb0) : nullptr, Ps, nullptr, nullptr, tid);
      __syncthreads();
      if (hp) {
        v4d acc[2][2];
        zero_acc(acc);
        for (int e = tk.po_beg; e < tk.po_end; ++e) {   // Ps is free until the pd loop
          const int32_t pa = pairs[2 * e], pb = pairs[2 * e + 1];
          const bool more = e + 1 < tk.po_end;
          d2v nv[2][8];
          int32_t na = -1, nb = -1;
          if (more) {
            na = pairs[2 * (e + 1)];
            nb = pairs[2 * (e + 1) + 1];
            tile_regs<SC1>(slot_ptr(b, na), nv[0], tid);
            if (nb != na) tile_regs<SC1>(slot_ptr(b, nb), nv[1], tid);
          }
          mfma_abt_acc(Qs, pb != pa ? Ps : Qs, w, l, acc);
          if (more) {
            __syncthreads();
            regs_tile(nv[0], Qs, tid);
            if (nb != na) regs_tile(nv[1], Ps, tid);
            __syncthreads();
          }
        }
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
          for (int tj = 0; tj < 2; ++tj)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) As[MFMA_ROW(w, l, ti, rr) * LD + MFMA_COL(w, l, tj)] -= acc[ti][tj][rr];
      }
    }
    if (tk.pd_end > tk.pd_beg) {
      __syncthreads();
      load_tile_lds_t<SC1>(slot_ptr(b, pairs[2 * tk.pd_beg]), Ps, tid);
      __syncthreads();
    }
    for (int e = tk.pd_beg; e < tk.pd_end; ++e) {
      const bool more = e + 1 < tk.pd_end;
      d2v nv[8];
      if (more) tile_regs<SC1>(slot_ptr(b, pairs[2 * (e + 1)]), nv, tid);
      diag_pending(accA, Ps, w, l);
      if (more) {
        __syncthreads();
        regs_tile(nv, Ps, tid);
        __syncthreads();
      }
    }
  }
  __syncthreads();
  TCLK(7, q, rtc());
  if (tid < T) S.vv[tid] = p.rk - ((S.rpart[0][tid] + S.rpart[1][tid]) + (S.rpart[2][tid] + S.rpart[3][tid]));
  // (2) pending diagonal update: block (0,0) by wave 0, blocks (0,v) by
  // waves v into the second exchange buffer (free until step 1), so wave 0
  // starts factoring after 16 MFMAs instead of 64
  const bool dp = p.fast && p.pd >= 0, op = p.fast && p.qa >= 0;
  if (dp) {
    if (w == 0) {
      accA[0] = pend_block(accA[0], Ps, 0, 0, l);
    } else {
      const v4d z = pend_block(v4d{0.0, 0.0, 0.0, 0.0}, Ps, 0, w, l);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) S.Xch[4 * 256 + w * 256 + rr * 64 + l] = z[rr];
    }
    __syncthreads();
    if (w == 0) {
#pragma unroll
      for (int TJ = 1; TJ < 4; ++TJ)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) accA[TJ][rr] += S.Xch[4 * 256 + TJ * 256 + rr * 64 + l];
    }
  }
  // this wave's own diagonal blocks (w, TJ >= w), before it factors
  auto diagpend = [&]() {
    if (dp) {
#pragma unroll
      for (int TJ = 1; TJ < 4; ++TJ)
        if (TJ >= w) accA[TJ] = pend_block(accA[TJ], Ps, w, TJ, l);
    }
  };
  TCLK(2, q, rtc());
  if (own) {
    // the own pair's second operand L(k,c): the first one or the pending
    // diagonal operand (Ps, read only before it is overwritten)
    const double* Rop = p.rb == p.qa ? Qs : Ps;
    auto chunk = [&](int c) {   // As(w, c) -= Q(w, :) R(c, :)^T, all 64 k in order
      if (!op) return;
      v4d tot = v4d{0.0, 0.0, 0.0, 0.0};   // one accumulator chain (as pend_block)
#pragma unroll
      for (int K = 0; K < 4; ++K) {
        const Kq a = ld_kq(Qs + (16 * w + li) * LD, K, lk), bq = ld_kq(Rop + (16 * c + li) * LD, K, lk);
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) tot = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s4], bq[s4], tot, 0, 0, 0);
      }
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) As[ACC_ROW(w, l, rr) * LD + ACC_COL(c, l)] -= tot[rr];
    };
    v4d XT[4];
    factor_own(accA, XT, w, l, S, diagpend, chunk, q, seq);
    __syncthreads();   // y_3 (wave 1, after the last barrier)
    TCLK(3, q, rtc());
    TCLK(8, q, rtc());
    TCLK(9, q, rtc());
    // L(i,k) row block w into As (its own rows, row-major), contribution
    // L(i,k) y_k of its rows from registers
    double cp = 0.0;
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        As[(16 * w + li) * LD + 16 * c + lk + 4 * r] = XT[c][r];
        cp += XT[c][r] * S.yv[16 * c + lk + 4 * r];
      }
    cp = sum_groups(cp);
    TCLK(10, q, rtc());
    // coalesced 16-byte stores of the 16 rows (write-through in the dataflow kernel)
    double* dst = slot_ptr(b, tk.dst);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, T * T * 8, 0x00020000);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = l + 64 * i, row = 16 * w + (e >> 5), c2 = 2 * (e & 31);
      const d2v v = d2v{As[row * LD + c2], As[row * LD + c2 + 1]};
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) int, v), rs,
                                             (row * T + c2) * 8, 0, SC1 ? 16 : 0);
    }
    TCLK(11, q, rtc());
    if (lk == 0) gst<SC1>(contrib + static_cast<int64_t>(tk.dst) * T + 16 * w + li, cp);
    return;
  }
  // the diagonal task: L_kk^-1 for the backward substitution, y_k
  v4d accX[4];
#pragma unroll
  for (int TJ = 0; TJ < 4; ++TJ)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) accX[TJ][rr] = ACC_ROW(w, l, rr) == ACC_COL(TJ, l) ? 1.0 : 0.0;
  auto idle = [&](int KB) {
    if (KB == 0) diagpend();
  };
  const bool ok = factor_tile_blk(accA, accX, w, l, S.Xch, &S.rpart[w][0], idle, q);
  TCLK(3, q, rtc());
  if (!ok && tid == 0) *fail = 1;
  double yp[4];
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) yp[rr] = 0.0;
#pragma unroll
  for (int TJ = 0; TJ < 4; ++TJ) {
    const double vj = S.vv[16 * TJ + li];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr)
      if (TJ <= w) yp[rr] += accX[TJ][rr] * vj;
  }
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) yp[rr] = sum16(yp[rr]);
  double* dst = Linv + static_cast<int64_t>(tk.k) * T * T;
#pragma unroll
  for (int TJ = 0; TJ < 4; ++TJ)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) dst[ACC_ROW(w, l, rr) * T + ACC_COL(TJ, l)] = accX[TJ][rr];
  if (li == 0) {
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) y[static_cast<int64_t>(tk.k) * T + ACC_ROW(w, l, rr)] = yp[rr];
  }
}

__global__ __launch_bounds__(256) void k_tasks(TileDev b, const TileTask* __restrict__ tasks,
                                               const int32_t* __restrict__ pairs, double* __restrict__ Linv,
                                               const double* __restrict__ r, double* __restrict__ contrib,
                                               double* __restrict__ y, int* fail) {
  __shared__ TaskLds S;
  const TileTask tk = tasks[blockIdx.x];
  const int tid = threadIdx.x;
  if (tid < 4) S.flagA[tid] = S.flagB[tid] = S.yflag[tid] = 0;   // seen after panel_task's first barrier
  if (tk.kind == 1) {
    run_update<false>(b, tk, pairs, S.Qs, S.Ps, tid, tid >> 6, tid & 63);
    return;
  }
  const PanelPre p = panel_prefetch(b, tk, pairs, r, tid >> 6, tid & 63);
  panel_task<false>(b, tk, pairs, p, Linv, contrib, y, fail, S);
}

// update tasks of a wide level: dst -= sum A B^T, with only the two
// operand tiles in LDS (two workgroups per CU)
__global__ __launch_bounds__(256) void k_updates(TileDev b, const TileTask* __restrict__ tasks,
                                                 const int32_t* __restrict__ pairs) {
  __shared__ double Qs[T * LD];
  __shared__ double Rs[T * LD];
  const TileTask tk = tasks[blockIdx.x];
  const int tid = threadIdx.x;
  run_update<false>(b, tk, pairs, Qs, Rs, tid, tid >> 6, tid & 63);
}

// The whole factorisation (and forward substitution) in one launch, as a
// dataflow over the same tasks: one resident workgroup per CU takes tasks in
// schedule order from a global queue, waits until every slot the task reads
// or writes has received the writes the level schedule puts before it
// (per-slot write counters, Plan::fdep), runs it, and publishes its slot
// (sc1 stores drained, then the counter bumped). A task only waits for
// tasks earlier in the queue, which were taken by running workgroups, so
// the launch cannot deadlock whatever the residency. Waits are bounded: a
// timeout sets bit 2 of *fail and the task still publishes, so the grid
// drains and the step is rejected.
constexpr int kSpinLimitF = 1 << 22;


__global__ __launch_bounds__(256) void k_factor_persist(TileDev b, const TileTask* __restrict__ tasks, int ntasks,
                                                        const int32_t* __restrict__ pairs,
                                                        const int32_t* __restrict__ dep_start,
                                                        const int32_t* __restrict__ dep,
                                                        const int32_t* __restrict__ order, unsigned* wcnt,
                                                        unsigned* queue, double* __restrict__ Linv,
                                                        const double* __restrict__ r, double* __restrict__ contrib,
                                                        double* __restrict__ y, int* fail) {
  __shared__ TaskLds S;
  __shared__ int s_q;
  const int tid = threadIdx.x;
  const int w = tid >> 6, l = tid & 63;
  if (tid < 4) S.flagA[tid] = S.flagB[tid] = S.yflag[tid] = 0;   // tasks flag with qpos + 1
  for (;;) {
    if (tid == 0) s_q = static_cast<int>(__hip_atomic_fetch_add(queue, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    __syncthreads();
    const int qpos = __builtin_amdgcn_readfirstlane(s_q);
    if (qpos >= ntasks) break;
    const int q = order[qpos];   // task id (schedule order); clocks and dependencies are per id
    const TileTask tk = tasks[q];
    TCLK(0, q, rtc());
    TCLK(5, q, blockIdx.x);
    PanelPre p;
    int32_t upa = -1, upb = -1;   // an update's first operand pair
    if (tk.kind == 0) {
      p = panel_prefetch(b, tk, pairs, r, w, l);
    } else if (tk.po_end > tk.po_beg) {
      upa = pairs[2 * tk.po_beg];
      upb = pairs[2 * tk.po_beg + 1];
    }
    // Dependencies in two classes: the pending operand tiles (a panel's
    // pending pairs, an update's first pair), whose producers are usually
    // the last to finish, and the rest. The task loads what the rest guards
    // while wave 0 still waits for the operands (late()).
    int32_t o0 = -1, o1 = -1, o2 = -1;
    if (tk.kind == 0) {
      if (p.fast) {
        o0 = p.pd;
        o1 = p.qa;
        o2 = p.rb;
      }
    } else {
      o0 = upa;
      o1 = upb;
    }
    const bool split = o0 >= 0 || o1 >= 0;
    auto wait_deps = [&](int cls) {   // cls 0: not an operand slot, 1: an operand slot, 2: all
      if (w != 0) return;
      bool ok = true;
      for (int j = dep_start[q] + l; j < dep_start[q + 1]; j += 64) {
        const int32_t sl = dep[2 * j];
        const int c1 = (sl == o0 || sl == o1 || sl == o2) ? 1 : 0;
        if (cls != 2 && c1 != cls) continue;
        const unsigned* c = wcnt + sl;
        const unsigned need = static_cast<unsigned>(dep[2 * j + 1]);
        int spins = 0;
        while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
          if (++spins > kSpinLimitF) { ok = false; break; }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      if (!ok) atomicOr(fail, 4);
    };
    wait_deps(split ? 0 : 2);
    __syncthreads();
    TCLK(1, q, rtc());
    auto late = [&]() {
      if (split) {
        wait_deps(1);
        __syncthreads();
      }
    };
    if (tk.kind == 1) run_update<true>(b, tk, pairs, S.Qs, S.Ps, tid, w, l, upa, upb, late);
    else panel_task<true>(b, tk, pairs, p, Linv, contrib, y, fail, S, q, late, qpos + 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    TCLK(4, q, rtc());
    if (tid == 0 && (tk.kind == 1 || tk.i != tk.k))
      __hip_atomic_fetch_add(wcnt + tk.dst, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// one level of the backward substitution,
//   x_k = L_kk^-T (y_k - sum_i L(i,k)^T x_i),
// with every column's entries split over workgroups of <= back_part_tiles
// tiles (BackPart). A workgroup sums L(i,k)^T x_i over its tiles (lane =
// column of the tile, 4 row groups, all loads of a tile issued together).
// A column with one part finishes directly. Otherwise each part stores its
// partial sum, releases it (agent-scope fence) and bumps the column's
// arrival counter; the last part acquires, adds the partials in part order
// (deterministic), applies L_kk^-T and re-arms the counter.
constexpr int kBackThreads = 256;
__global__ __launch_bounds__(kBackThreads) void k_back(TileDev b, const BackPart* __restrict__ parts,
                                                       const int32_t* __restrict__ ent,
                                                       const double* __restrict__ Linv,
                                                       const double* __restrict__ y, double* __restrict__ x,
                                                       double* __restrict__ partials, int* __restrict__ arrive) {
  constexpr int NP = kBackThreads / T;
  __shared__ double part[NP][T];
  __shared__ double rv[T];
  __shared__ int last;
  const BackPart pt = parts[blockIdx.x];
  const int tid = threadIdx.x, c = tid & (T - 1), q = tid >> 6;
  double s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int e = pt.beg; e < pt.end; ++e) {
    const double* L = slot_ptr(b, ent[2 * e]);
    const double* xi = x + static_cast<int64_t>(ent[2 * e + 1]) * T;
    double lv[16], xv[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      lv[m] = L[(q + NP * m) * T + c];
      xv[m] = xi[q + NP * m];
    }
#pragma unroll
    for (int m = 0; m < 16; ++m) s[m & 7] += lv[m] * xv[m];
  }
  part[q][c] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  double sum = 0.0;
  if (tid < T) sum = (part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid]);
  if (pt.nparts > 1) {
    if (tid < T) partials[static_cast<int64_t>(pt.pbase + pt.part) * T + tid] = sum;
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      const int prev = __hip_atomic_fetch_add(arrive + pt.k, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = prev == pt.nparts - 1;
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        arrive[pt.k] = 0;
      }
    }
    __syncthreads();
    if (!last) return;
    if (tid < T) {
      sum = 0.0;
      for (int p = 0; p < pt.nparts; ++p) sum += partials[static_cast<int64_t>(pt.pbase + p) * T + tid];
    }
  }
  if (tid < T) rv[tid] = y[static_cast<int64_t>(pt.k) * T + tid] - sum;
  __syncthreads();
  // x_k[c] = sum_{m >= c} Linv[m][c] rv[m]
  const double* Li = Linv + static_cast<int64_t>(pt.k) * T * T;
  double t = 0.0;
#pragma unroll 4
  for (int m = q; m < T; m += NP)
    if (m >= c) t += Li[m * T + c] * rv[m];
  part[q][c] = t;
  __syncthreads();
  if (tid < T)
    x[static_cast<int64_t>(pt.k) * T + tid] = (part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid]);
}

// The whole backward substitution in one launch: workgroup b runs part b of
// the parts listed in backward-level order (a topological order). A part
// waits until the columns it reads are done in this solve (done[i] ==
// epoch). The launcher only uses it when every part can be resident at
// once, so each wait is for a workgroup that is already running. Every wait
// is still bounded: after ~2^22 polls the part sets bit 1 of *fail and
// gives up, so a broken schedule ends in an error, not a hang.
// Hand-offs follow cdna_hip_programming.md Guideline 16, R1. The payloads
// (x_k and the partial sums) are written with agent-scope relaxed atomic
// stores (write-through sc1) and drained (vmcnt(0)) by every storing wave
// before one lane stores the flag or adds to the counter. Consumers read
// them only with agent-scope atomic loads (sc1, to registers), so neither a
// release nor an acquire fence is needed. Operands that no workgroup of
// this launch writes (L tiles, L^-1, y) are fetched before the wait.
constexpr int kSpinLimit = 1 << 22;

__device__ __forceinline__ double ld_sc1(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kBackThreads) void k_back_persist(TileDev b, const BackPart* __restrict__ parts,
                                                               const int32_t* __restrict__ ent,
                                                               const double* __restrict__ Linv,
                                                               const double* __restrict__ y, double* x,
                                                               double* partials, int* arrive, unsigned* done,
                                                               unsigned epoch, int* fail) {
  constexpr int NP = kBackThreads / T;
#ifndef DYNOHIP_BACK_CH
#define DYNOHIP_BACK_CH 4
#endif
  constexpr int CH = DYNOHIP_BACK_CH;  // entries per chunk; the first chunk is fetched before the wait
  __shared__ double part[NP][T];
  __shared__ double rv[T];
  __shared__ double xs[CH][T];
  __shared__ int last, abort_;
  const BackPart pt = parts[blockIdx.x];
  const int tid = threadIdx.x, c = tid & (T - 1), q = tid >> 6;
  const int ne = pt.end - pt.beg;
  // (1) prefetch what does not depend on other columns
  double lv[CH][16];
#pragma unroll
  for (int j = 0; j < CH; ++j)
    if (j < ne) {
      const double* L = slot_ptr(b, ent[2 * (pt.beg + j)]);
#pragma unroll
      for (int m = 0; m < 16; ++m) lv[j][m] = L[(q + NP * m) * T + c];
    }
  const double* Li = Linv + static_cast<int64_t>(pt.k) * T * T;
  double li[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) li[m] = Li[(q + NP * m) * T + c];
  const double yk = tid < T ? y[static_cast<int64_t>(pt.k) * T + tid] : 0.0;
  // (2) wait for the columns this part reads (one lane polls, relaxed)
  if (tid == 0) {
    int ok = 1;
    for (int e = pt.beg; e < pt.end && ok; ++e) {
      const unsigned* d = done + ent[2 * e + 1];
      int spins = 0;
      while (__hip_atomic_load(d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
        if (++spins > kSpinLimit) { ok = 0; break; }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    if (!ok) atomicOr(fail, 2);
    abort_ = !ok;
  }
  __syncthreads();
  if (abort_) return;
  // (3) x of the rows read, sc1 loads (lane-varying: vector path), chunk
  // by chunk; later chunks' L tiles are loaded after the wait
  double s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int j0 = 0; j0 < ne; j0 += CH) {
    if (j0 > 0) {
      __syncthreads();
#pragma unroll
      for (int j = 0; j < CH; ++j)
        if (j0 + j < ne) {
          const double* L = slot_ptr(b, ent[2 * (pt.beg + j0 + j)]);
#pragma unroll
          for (int m = 0; m < 16; ++m) lv[j][m] = L[(q + NP * m) * T + c];
        }
    }
    if (tid < min(CH, ne - j0) * T)
      xs[tid >> 6][c] = ld_sc1(x + static_cast<int64_t>(ent[2 * (pt.beg + j0 + (tid >> 6)) + 1]) * T + c);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < CH; ++j)
      if (j0 + j < ne) {
#pragma unroll
        for (int m = 0; m < 16; ++m) s[m & 7] += lv[j][m] * xs[j][q + NP * m];
      }
  }
  part[q][c] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  double sum = 0.0;
  if (tid < T) sum = (part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid]);
  if (pt.nparts > 1) {
    if (tid < T) st_sc1(partials + static_cast<int64_t>(pt.pbase + pt.part) * T + tid, sum);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const int prev = __hip_atomic_fetch_add(arrive + pt.k, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = prev == pt.nparts - 1;
      if (last) __hip_atomic_store(arrive + pt.k, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last) return;
    if (tid < T) {
      sum = 0.0;
      for (int p = 0; p < pt.nparts; ++p) sum += ld_sc1(partials + static_cast<int64_t>(pt.pbase + p) * T + tid);
    }
  }
  if (tid < T) rv[tid] = yk - sum;
  __syncthreads();
  // x_k[c] = sum_{m >= c} Linv[m][c] rv[m]
  double t = 0.0;
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const int row = q + NP * m;
    if (row >= c) t += li[m] * rv[row];
  }
  part[q][c] = t;
  __syncthreads();
  if (tid < T) {
    st_sc1(x + static_cast<int64_t>(pt.k) * T + tid, (part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid]));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tid == 0) __hip_atomic_store(done + pt.k, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// The backward substitution in one launch with the hand-offs on the data
// itself (the default; k_back_persist above is the flag form). Before each
// solve the solution x and the part partials are filled with kBackSent, a
// signalling-NaN pattern that no arithmetic produces (an FP64 operation
// returns quiet NaNs), so a consumer knows a value is this solve's by seeing
// anything else. Per level that is one memory round trip instead of the
// flag form's drain, flag poll and then payload load, and a column split
// into parts needs no arrival counter:
//   * a part polls the x rows of its entries (sc1 loads, each lane its own
//     element) with its L tiles and L_kk^-1 fetched before;
//   * a column of one part solves x_k at once;
//   * otherwise parts 1.. store their partial sums and leave, and part 0
//     polls them and adds them in part order (the same order and operations
//     as the counter form: the results are bit-identical), then solves x_k.
// Every part is resident (the same kBackPersistMax bound), so each wait is
// for a running workgroup. A wait that times out (~2^22 polls) sets bit 1 of
// *fail and the part stores a quiet NaN instead, so the chain drains quickly
// and the step is rejected.
constexpr uint64_t kBackSent = 0xFFF4DEADBEEFCAFEull;
__device__ __forceinline__ bool back_sent(double v) { return __builtin_bit_cast(uint64_t, v) == kBackSent; }
// an sc1 load of *p repeated until it is not the sentinel (false on timeout)
__device__ __forceinline__ bool poll_value(const double* p, double& v) {
  v = ld_sc1(p);
  int spins = 0;
  while (back_sent(v)) {
    if (++spins > kSpinLimit) return false;
    __builtin_amdgcn_s_sleep(1);
    v = ld_sc1(p);
  }
  return true;
}

__global__ __launch_bounds__(kBackThreads) void k_back_poll(TileDev b, const BackPart* __restrict__ parts,
                                                            const int32_t* __restrict__ ent,
                                                            const double* __restrict__ Linv,
                                                            const double* __restrict__ y, double* x,
                                                            double* partials, int* fail) {
  constexpr int NP = kBackThreads / T;
  constexpr int CH = DYNOHIP_BACK_CH;
  __shared__ double part[NP][T];
  __shared__ double rv[T];
  __shared__ double xs[CH][T];
  const BackPart pt = parts[blockIdx.x];
  const int tid = threadIdx.x, c = tid & (T - 1), q = tid >> 6;
  const int ne = pt.end - pt.beg;
  int bad = 0;   // this thread's waits timed out
  // (1) what does not depend on other columns
  double lv[CH][16];
#pragma unroll
  for (int j = 0; j < CH; ++j)
    if (j < ne) {
      const double* L = slot_ptr(b, ent[2 * (pt.beg + j)]);
#pragma unroll
      for (int m = 0; m < 16; ++m) lv[j][m] = L[(q + NP * m) * T + c];
    }
  const bool solver = pt.nparts == 1 || pt.part == 0;
  double li[16];
  if (solver) {
    const double* Li = Linv + static_cast<int64_t>(pt.k) * T * T;
#pragma unroll
    for (int m = 0; m < 16; ++m) li[m] = Li[(q + NP * m) * T + c];
  }
  const double yk = (solver && tid < T) ? y[static_cast<int64_t>(pt.k) * T + tid] : 0.0;
  // (2) the x rows of the entries, chunk by chunk, each element polled
  double s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int j0 = 0; j0 < ne; j0 += CH) {
    if (j0 > 0) {
      __syncthreads();
#pragma unroll
      for (int j = 0; j < CH; ++j)
        if (j0 + j < ne) {
          const double* L = slot_ptr(b, ent[2 * (pt.beg + j0 + j)]);
#pragma unroll
          for (int m = 0; m < 16; ++m) lv[j][m] = L[(q + NP * m) * T + c];
        }
    }
    if (tid < min(CH, ne - j0) * T) {
      double v;
      if (!poll_value(x + static_cast<int64_t>(ent[2 * (pt.beg + j0 + (tid >> 6)) + 1]) * T + c, v)) bad = 1;
      xs[tid >> 6][c] = v;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < CH; ++j)
      if (j0 + j < ne) {
#pragma unroll
        for (int m = 0; m < 16; ++m) s[m & 7] += lv[j][m] * xs[j][q + NP * m];
      }
  }
  part[q][c] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  double sum = 0.0;
  if (tid < T) sum = (part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid]);
  if (pt.nparts > 1) {
    if (!solver) {
      // hand the partial to part 0 (a quiet NaN after a timed-out wait)
      bad = __syncthreads_or(bad);
      if (tid < T) st_sc1(partials + static_cast<int64_t>(pt.pbase + pt.part) * T + tid, bad ? __builtin_nan("") : sum);
      if (tid == 0 && bad) atomicOr(fail, 2);
      return;
    }
    if (tid < T) {
      const double own = sum;
      sum = 0.0;
      for (int p = 0; p < pt.nparts; ++p) {
        double v = own;
        if (p > 0 && !poll_value(partials + static_cast<int64_t>(pt.pbase + p) * T + tid, v)) bad = 1;
        sum += v;
      }
    }
  }
  if (tid < T) rv[tid] = yk - sum;
  __syncthreads();
  // x_k[c] = sum_{m >= c} Linv[m][c] rv[m]
  double t = 0.0;
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const int row = q + NP * m;
    if (row >= c) t += li[m] * rv[row];
  }
  part[q][c] = t;
  bad = __syncthreads_or(bad);
  if (tid < T) {
    const double xv = (part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid]);
    st_sc1(x + static_cast<int64_t>(pt.k) * T + tid, bad ? __builtin_nan("") : xv);
  }
  if (tid == 0 && bad) atomicOr(fail, 2);
}

// ---- small reduced systems (<= kSmallNT tiles): one workgroup, dataflow ---
// The sliding-window solves (backend.flags: 10-frame windows) have reduced
// systems of at most four tiles (16 blocks of 16), where the tile DAG is a
// chain of four dependent panels with a global-memory hand-off between each,
// and the backward substitution four more. k_small_solve does the whole solve
// in one workgroup of 16 waves, the position-ordered matrix (upper triangle,
// A = U^T U) resident in registers as 16x16 blocks in MFMA accumulator layout,
// the waves handing blocks to each other through LDS flags (no barriers after
// the first):
//   * wave 0 factors the diagonal blocks one after the other (factor16: U_KK
//     and W_K = U_KK^-1), publishes W_K and y_K = W_K^T r_K, then forms the
//     superdiagonal block U[K][K+1] = W_K^T A[K][K+1] itself and with it the
//     next diagonal block D(K+1) - U^T U and r_{K+1} - U^T y_K, so the chain
//     of diagonal blocks never leaves the wave;
//   * wave J (1..15) keeps D(J), A[J-1][J] and r_J up to date with the steps
//     before J-1 and hands them to wave 0 after step J-2 (before wave 0 needs
//     them, while it factors D(J-1));
//   * the other 105 blocks (I, J >= I+2) are dealt over waves 1..15, seven
//     each (eight spill registers to scratch); at step K the owners of row K form
//     U[K][J] = W_K^T A[K][J] into an LDS ring of two rows, and every owner of
//     a block below takes A[I][J] -= U[K][I]^T U[K][J] as the operands come
//     out. A ring row is rewritten only once every wave is done with the step
//     that read it (per-wave progress counters).
// The forward substitution rides along (r_I updated with the blocks), and the
// backward substitution x_K = W_K (y_K - sum_{J>K} U[K][J] x_J) uses the U
// blocks where they were formed: each owner adds U[K][J] x_J to an LDS slot
// as soon as x_J is out (its blocks in descending J, the order in which the
// x_J come), and wave 0 sums the slots of row K in J order. Results match the
// tile DAG's up to the summation order.
// Measured on the C2 stream's 10-frame windows (four tiles, 95 % of the
// 16x16 blocks nonzero after fill): 72 us per solve (HIP events) against the
// DAG's 57 + 13 us, so it stays opt-in (DYNOHIP_SMALL_SOLVE=1). The bound is
// the one CU's f64 MFMA rate: ~3200 MFMAs at ~100 cycles each per SIMD
// (unchanged with half the LDS operand reads), the early steps throughput-
// bound while wave 0 waits for its hand-overs, and the factoring wave slowed
// from 3.0k to 5-7k cycles per block while the waves on its SIMD issue
// MFMAs; the backward chain ~1.8k cycles per block (tools/small_clock.py).
constexpr int kSmallNB = 4 * kSmallNT;   // 16x16 blocks per dimension
constexpr int kSW = 16;                  // waves
constexpr int kSReg = 7;                 // off-band blocks per wave (at most)
constexpr int kSRing = 2;                // rows of U in flight
constexpr int kSRow = kSmallNB - 2;      // off-band blocks of a U row (J >= K + 2)
constexpr int kSStage = 16 * 18;         // a wave's staging rows at the start (in the ring)
static_assert(kSmallNB == 16, "the small solve's block deal is for 16 blocks");

struct SmallDeal {
  int8_t I[kSW][kSReg], J[kSW][kSReg];
};
// off-band blocks (I, J >= I + 2) by rows, round-robin over the waves (those
// on wave 0's SIMD, 4, 8 and 12, last in the cycle); each wave's blocks in
// descending J (then I) order
constexpr SmallDeal small_deal() {
  SmallDeal d{};
  for (int w = 0; w < kSW; ++w)
    for (int s = 0; s < kSReg; ++s) d.I[w][s] = d.J[w][s] = -1;
  const int order[15] = {1, 2, 3, 5, 6, 7, 9, 10, 11, 13, 14, 15, 4, 8, 12};
  int cap[kSW] = {}, cnt[kSW] = {};
  for (int w = 1; w < kSW; ++w) cap[w] = kSReg;
  int c = 0;
  for (int I = 0; I < kSmallNB; ++I)
    for (int J = I + 2; J < kSmallNB; ++J) {
      while (cnt[order[c]] >= cap[order[c]]) c = (c + 1) % 15;
      const int w = order[c];
      d.I[w][cnt[w]] = static_cast<int8_t>(I);
      d.J[w][cnt[w]] = static_cast<int8_t>(J);
      ++cnt[w];
      c = (c + 1) % 15;
    }
  for (int w = 1; w < kSW; ++w)
    for (int a = 1; a < cnt[w]; ++a)
      for (int b = a; b > 0; --b) {
        const bool later = d.J[w][b] > d.J[w][b - 1] || (d.J[w][b] == d.J[w][b - 1] && d.I[w][b] > d.I[w][b - 1]);
        if (!later) break;
        const int8_t ti = d.I[w][b], tj = d.J[w][b];
        d.I[w][b] = d.I[w][b - 1];
        d.J[w][b] = d.J[w][b - 1];
        d.I[w][b - 1] = ti;
        d.J[w][b - 1] = tj;
      }
  return d;
}
__constant__ SmallDeal kSmallDeal = small_deal();

// a 16x16 block in LDS: every lane's (v0, v1) pair, then every lane's (v2,
// v3) pair: two conflict-free 16-byte accesses per lane
typedef double d2s __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void st_b2(double* p, const v4d& v, int l) {
  reinterpret_cast<d2s*>(p)[l] = d2s{v[0], v[1]};
  reinterpret_cast<d2s*>(p + 128)[l] = d2s{v[2], v[3]};
}
__device__ __forceinline__ v4d ld_b2(const double* p, int l) {
  const d2s a = reinterpret_cast<const d2s*>(p)[l], b = reinterpret_cast<const d2s*>(p + 128)[l];
  return v4d{a[0], a[1], b[0], b[1]};
}

struct SmallLds {
  double Ws[kSmallNB][256];            // W_K
  double Usd[kSmallNB - 1][256];       // U[K][K+1]
  double ring[kSRing][kSRow][256];     // U[K][J], J >= K + 2, at [K % kSRing][J - K - 2]
  double hb[2][2][256];                // D(J), A[J-1][J] handed to wave 0 (buffer J & 1)
  double hr[2][16];                    // r_J handed over
  double rs[kSmallNB][16];             // r_K (wave 0's, for the column form)
  double ys[kSmallNB][16];             // y_K
  double xs[kSmallNB][16];             // x_K
  double pb[kSmallNB * (kSmallNB - 1) / 2][16];   // U[K][J] x_J, J > K (upper-triangle index)
  double dscr[16];
  int wf[kSmallNB], yf[kSmallNB], sf[kSmallNB], xf[kSmallNB], prc[kSmallNB];
  int uf[kSRing][kSmallNB];
  int hf[2];
  int urc[kSRing];                     // blocks published into each ring row (cumulative)
  int prog[kSW];
  int abort;
};
static_assert(sizeof(SmallLds) <= 160 * 1024, "the small solve's LDS");
static_assert(kSW * kSStage <= kSRing * kSRow * 256, "the staging rows fit in the ring");

// upper-triangle index of (K, J), K < J
__device__ __forceinline__ int small_ut(int K, int J) { return K * (2 * kSmallNB - K - 1) / 2 + (J - K - 1); }

// The waits of the small solve are bounded: a wait that polls 2^22 times
// (~0.3 s) without its value sets S.abort, every later wait returns at once,
// and wave 0 reports the solve as failed (no hang on a broken hand-off).
constexpr int kSmallPolls = 1 << 22;
__device__ __forceinline__ int lds_ld(const int* p) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ void small_wait(const int* f, int v, int* abort) {
  for (int n = 0; n < kSmallPolls; ++n) {
    if (lds_ld(f) == v) return;
    __builtin_amdgcn_s_sleep(1);   // (the polls of 15 waves would crowd the LDS)
    if ((n & 63) == 63 && lds_ld(abort)) return;
  }
  lds_flag_set(abort, 1);
}
// until each of the 16 waves' progress counters is >= v
__device__ __forceinline__ void small_wait_prog(const int* prog, int v, int l, int* abort) {
  for (int n = 0; n < kSmallPolls; ++n) {
    const int p = __hip_atomic_load(prog + (l & 15), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (__all(p >= v)) return;
    __builtin_amdgcn_s_sleep(1);
    if ((n & 63) == 63 && lds_ld(abort)) return;
  }
  lds_flag_set(abort, 1);
}
// blocks published into ring row K % kSRing up to and including row K
__device__ __forceinline__ int small_ring_count(int K, int nb) {
  int c = 0;
  for (int j = K & 1; j <= K; j += 2) c += max(0, nb - j - 2);
  return c;
}

__global__ __launch_bounds__(kSW * 64) void k_small_solve(TileDev b, SmallMap m, const double* __restrict__ r,
                                                          double* __restrict__ x, int* fail) {
  __shared__ __attribute__((aligned(16))) SmallLds S;
  const int tid = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6), l = tid & 63;
  const int NT = b.NT, nb = 4 * NT;
  const int li = l & 15, g = l >> 4;
  if (tid < kSmallNB) {
    S.wf[tid] = S.yf[tid] = S.sf[tid] = S.xf[tid] = S.prc[tid] = 0;
    S.prog[tid] = tid == 0 ? 1 << 30 : 0;   // wave 0 reads no ring row
    for (int q = 0; q < kSRing; ++q) S.uf[q][tid] = 0;
    if (tid < kSRing) S.urc[tid] = 0;
    if (tid < 2) S.hf[tid] = 0;
    if (tid == 0) S.abort = 0;
  }
  __syncthreads();
  const v4d zero = v4d{0.0, 0.0, 0.0, 0.0};
  // Block (I, J), I <= J, of the position-ordered matrix (zero where no tile
  // is stored, or when !use): its 16x16 source region read row by row with
  // coalesced 16-byte loads (raw_load; branch-free, so a wave's loads all go
  // out together), then turned into accumulator layout through the wave's own
  // LDS staging rows (unstage; transposed for a block of an off-diagonal
  // tile, which stores A[I][J]^T). Direct accumulator-layout loads of the
  // transposed blocks touch 16 rows per instruction and kept the last waves
  // waiting ~10 us for their blocks.
  struct RawBlk {
    d2s h0, h1;
    bool tr, present;
  };
  auto raw_load = [&](int I, int J, bool use) {
    const int Ic = use ? I : 0, Jc = use ? J : 0;
    const int p = Ic >> 2, q = Jc >> 2, sl = m.slot[p][q];
    RawBlk rb;
    rb.present = use && sl >= 0;
    rb.tr = p != q;
    const double* t = slot_ptr(b, rb.present ? sl : 0);
    const int br = rb.tr ? 16 * (Jc & 3) : 16 * (Ic & 3), bc = rb.tr ? 16 * (Ic & 3) : 16 * (Jc & 3);
    const d2s* src = reinterpret_cast<const d2s*>(t + (br + (l >> 3)) * T + bc + 2 * (l & 7));
    rb.h0 = src[0];
    rb.h1 = src[4 * T];   // eight rows down
    return rb;
  };
  double* stg = &S.ring[0][0][0] + w * kSStage;
  auto unstage = [&](const RawBlk& rb) {
    reinterpret_cast<d2s*>(stg + (l >> 3) * 18)[l & 7] = rb.h0;
    reinterpret_cast<d2s*>(stg + ((l >> 3) + 8) * 18)[l & 7] = rb.h1;
    v4d v;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) v[rr] = rb.tr ? stg[li * 18 + g + 4 * rr] : stg[(g + 4 * rr) * 18 + li];
    return rb.present ? v : zero;
  };
  // r_I[li] (every row group)
  auto load_r = [&](int I) { return r[static_cast<int64_t>(m.ord[I >> 2]) * T + 16 * (I & 3) + li]; };
  // (Y^T v)[li] for a block Y and a vector v in LDS (v[g + 4rr] read here)
  auto tmatvec = [&](const v4d& Y, const double* v) {
    double p = 0.0;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) p = __builtin_fma(Y[rr], v[g + 4 * rr], p);
    return sum_groups(p);
  };

  // ---- the matrix into registers: wave 0 D(0) and r_0; wave J its
  // off-band blocks and its band D(J), A[J-1][J], r_J ----
  int bI[kSReg], bJ[kSReg];
  v4d A[kSReg];
  const int J = w;
  const bool band = w > 0 && J < nb;
  v4d Dp, Ap;
  double rp;
  {
    RawBlk rb[kSReg];
#pragma unroll
    for (int s = 0; s < kSReg; ++s) {
      bI[s] = w > 0 ? kSmallDeal.I[w][s] : -1;
      bJ[s] = w > 0 ? kSmallDeal.J[w][s] : -1;
      if (bJ[s] >= nb) bI[s] = -1;   // outside this system (or no block)
      rb[s] = raw_load(bI[s], bJ[s], bI[s] >= 0);
    }
    const RawBlk rd = raw_load(J, J, w == 0 ? nb > 0 : band), ra = raw_load(J - 1, J, band);
    rp = (w == 0 ? nb > 0 : band) ? load_r(J) : 0.0;
#pragma unroll
    for (int s = 0; s < kSReg; ++s) A[s] = unstage(rb[s]);
    Dp = unstage(rd);
    Ap = unstage(ra);
  }
  __syncthreads();   // the staging rows (ring) free
  TCLKW(28, w);
  if (w == 0) {
    // ---- the chain of diagonal blocks ----
    bool ok = true;
    v4d D = Dp;
    double rk = rp;
    for (int K = 0; K < nb; ++K) {
      TCLKW(20, K);
      if (g == 0) S.rs[K][li] = rk;
      v4d Wm;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) Wm[rr] = (g + 4 * rr == li) ? 1.0 : 0.0;
      factor16(D, Wm, l, ok, &S.dscr[0]);
      st_b2(&S.Ws[K][0], Wm, l);
      lds_flag_set(&S.wf[K], 1);
      TCLKW(21, K);
      if (K + 1 < nb) {
        const int hbuf = (K + 1) & 1;
        small_wait(&S.hf[hbuf], K + 1, &S.abort);
        TCLKW(22, K);
        const v4d Dn = ld_b2(&S.hb[hbuf][0][0], l), An = ld_b2(&S.hb[hbuf][1][0], l);
        const double rn = S.hr[hbuf][li];
        const v4d U = mfma_tn(Wm, An, zero, false);
        st_b2(&S.Usd[K][0], U, l);
        lds_flag_set(&S.sf[K], 1);
        D = mfma_tn(U, U, Dn, true);
        const double yk = tmatvec(Wm, &S.rs[K][0]);
        if (g == 0) S.ys[K][li] = yk;
        lds_flag_set(&S.yf[K], 1);
        rk = rn - tmatvec(U, &S.ys[K][0]);
        TCLKW(23, K);
      } else {
        const double yk = tmatvec(Wm, &S.rs[K][0]);
        if (g == 0) S.ys[K][li] = yk;
        lds_flag_set(&S.yf[K], 1);
      }
    }
    // ---- backward: x_K = W_K (y_K - sum_{J > K} U[K][J] x_J) ----
    for (int K = nb - 1; K >= 0; --K) {
      const v4d Wk = ld_b2(&S.Ws[K][0], l);
      const v4d Um = ld_b2(&S.Usd[K >= 1 ? K - 1 : 0][0], l);
      const double yk = S.ys[K][li];
      small_wait(&S.prc[K], max(0, nb - K - 2), &S.abort);
      double t = yk;
      for (int J = K + 1; J < nb; ++J) t -= S.pb[small_ut(K, J)][li];
      double xr[4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) xr[rr] = sum16(Wk[rr] * t);
      if (li == 0) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          S.xs[K][g + 4 * rr] = xr[rr];
          x[static_cast<int64_t>(m.ord[K >> 2]) * T + 16 * (K & 3) + g + 4 * rr] = xr[rr];
        }
      }
      lds_flag_set(&S.xf[K], 1);
      TCLKW(24, K);
      if (K >= 1) {
        // the superdiagonal product U[K-1][K] x_K, for row K-1
        const double xk = S.xs[K][li];
        double pr[4];
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) pr[rr] = sum16(Um[rr] * xk);
        if (li == 0) {
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) S.pb[small_ut(K - 1, K)][g + 4 * rr] = pr[rr];
        }
      }
    }
    if ((!ok || lds_ld(&S.abort)) && l == 0) *fail = 1;
    TCLKW(29, w);
    return;
  }

  // ---- waves 1..15 ----
  // this wave's band: D(J), A[J-1][J], r_J for J = w, handed over after step J - 2
  auto hand_over = [&]() {
    const int hbuf = J & 1;
    st_b2(&S.hb[hbuf][0][0], Dp, l);
    st_b2(&S.hb[hbuf][1][0], Ap, l);
    if (g == 0) S.hr[hbuf][li] = rp;
    lds_flag_set(&S.hf[hbuf], J);
    TCLKW(27, J);
  };
  if (band && J == 1) hand_over();
  auto ring = [&](int K, int Jr) { return &S.ring[K % kSRing][Jr - K - 2][0]; };
  for (int K = 0; K < nb; ++K) {
    small_wait(&S.wf[K], 1, &S.abort);
    TCLKW(26, 16 * w + K);
    // (1) row K of U
    bool first = true;
#pragma unroll
    for (int s = 0; s < kSReg; ++s)
      if (bI[s] == K) {
        if (first) small_wait_prog(S.prog, K - kSRing + 1, l, &S.abort);   // ring row K % kSRing free
        first = false;
        const v4d Wk = ld_b2(&S.Ws[K][0], l);
        A[s] = mfma_tn(Wk, A[s], zero, false);
        st_b2(ring(K, bJ[s]), A[s], l);
        lds_flag_set(&S.uf[K % kSRing][bJ[s]], K + 1);
        if (l == 0) __hip_atomic_fetch_add(&S.urc[K % kSRing], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    // (2) the band blocks, handed to wave 0 after step J - 2
    if (band && K <= J - 2) {
      small_wait(&S.uf[K % kSRing][J], K + 1, &S.abort);
      const v4d Uj = ld_b2(ring(K, J), l);
      v4d Uj1;
      if (K == J - 2) {
        small_wait(&S.sf[K], 1, &S.abort);
        Uj1 = ld_b2(&S.Usd[K][0], l);
      } else {
        small_wait(&S.uf[K % kSRing][J - 1], K + 1, &S.abort);
        Uj1 = ld_b2(ring(K, J - 1), l);
      }
      Dp = mfma_tn(Uj, Uj, Dp, true);
      Ap = mfma_tn(Uj1, Uj, Ap, true);
      small_wait(&S.yf[K], 1, &S.abort);
      rp -= tmatvec(Uj, &S.ys[K][0]);
      if (K == J - 2) hand_over();
    }
    // (3) the trailing update of this wave's blocks below row K, once the
    // whole of row K is out
    bool below = false;
#pragma unroll
    for (int s = 0; s < kSReg; ++s) below = below || bI[s] > K;
    if (below) small_wait(&S.urc[K % kSRing], small_ring_count(K, nb), &S.abort);
#pragma unroll
    for (int s = 0; s < kSReg; ++s)
      if (bI[s] > K) {
        const int I = bI[s];
        v4d U1;
        if (I == K + 1) {
          small_wait(&S.sf[K], 1, &S.abort);
          U1 = ld_b2(&S.Usd[K][0], l);
        } else {
          U1 = ld_b2(ring(K, I), l);
        }
        A[s] = mfma_tn(U1, ld_b2(ring(K, bJ[s]), l), A[s], true);
      }
    lds_flag_set(&S.prog[w], K + 1);
    TCLKW(25, 16 * w + K);
  }
  // backward: U[I][J] x_J of this wave's blocks, in descending J
#pragma unroll
  for (int s = 0; s < kSReg; ++s)
    if (bI[s] >= 0) {
      small_wait(&S.xf[bJ[s]], 1, &S.abort);
      const double xj = S.xs[bJ[s]][li];
      double pr[4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) pr[rr] = sum16(A[s][rr] * xj);
      if (li == 0) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) S.pb[small_ut(bI[s], bJ[s])][g + 4 * rr] = pr[rr];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (l == 0) __hip_atomic_fetch_add(&S.prc[bI[s]], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  TCLKW(29, w);
}

}  // namespace

#ifdef DYNOHIP_TASK_CLOCK
extern "C" int dynohip_debug_task_clock(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tclk), sizeof(unsigned long long) * 32 * 32768) == hipSuccess ? n : -1;
}
#endif

void launch_tile_forward(const TileDev& b, const TileSchedDev& sd, const std::vector<int32_t>& flevel,
                         const std::vector<int32_t>& fpanels, double* Linv, const double* r, double* contrib,
                         double* y, int* fail, hipStream_t s, hipStream_t side, hipEvent_t ev_main,
                         hipEvent_t ev_side) {
  // a level is "wide" when its update tasks alone need more than one
  // round of the CUs (sd.wide_updates, default 256): they then run as
  // k_updates on the side stream
  const int ntasks = flevel.empty() ? 0 : flevel.back();
  if (sd.persistent_factor && ntasks > 0) {
    k_factor_persist<<<std::min(ntasks, sd.workers), 256, 0, s>>>(b, sd.ftask, ntasks, sd.pairs, sd.fdep_start, sd.fdep,
                                                                  sd.forder, sd.wcnt, sd.fqueue, Linv, r, contrib, y,
                                                                  fail);
  }
  for (size_t lv = 0; lv + 1 < flevel.size() && !sd.persistent_factor; ++lv) {
    const int n = flevel[lv + 1] - flevel[lv];
    const int np = fpanels[lv], nu = n - np;
    if (nu > 0 && nu > sd.wide_updates && side) {
      (void)hipEventRecord(ev_main, s);
      (void)hipStreamWaitEvent(side, ev_main, 0);
      if (np > 0) k_tasks<<<np, 256, 0, s>>>(b, sd.ftask + flevel[lv], sd.pairs, Linv, r, contrib, y, fail);
      k_updates<<<nu, 256, 0, side>>>(b, sd.ftask + flevel[lv] + np, sd.pairs);
      (void)hipEventRecord(ev_side, side);
      (void)hipStreamWaitEvent(s, ev_side, 0);
    } else if (n > 0) {
      k_tasks<<<n, 256, 0, s>>>(b, sd.ftask + flevel[lv], sd.pairs, Linv, r, contrib, y, fail);
    }
  }
}

void launch_tile_backward(const TileDev& b, const TileSchedDev& sd, const std::vector<int32_t>& blevel,
                          const double* Linv, const double* y, double* x, int* fail, hipStream_t s,
                          bool sentinel_filled) {
  const int nparts = blevel.empty() ? 0 : blevel.back();
  if (nparts > 0 && nparts <= kBackPersistMax && !sd.level_backward) {
    // past 512 parts (two per CU) not all are resident: the parts are in
    // backward-level (topological) order and each XCD dispatches its
    // workgroups in index order, so the lowest-indexed waiting part only ever
    // waits for a running one. k_back_poll reads "not written yet" as
    // kBackSent in x and the partials, so it runs only when the caller has
    // filled them for this solve (enqueue_try: the chain launch's ZeroDev.s);
    // otherwise the flag form, which needs no fill
    if (sd.back_poll && sentinel_filled)
      k_back_poll<<<nparts, kBackThreads, 0, s>>>(b, sd.bpart, sd.bent, Linv, y, x, sd.partials, fail);
    else
      k_back_persist<<<nparts, kBackThreads, 0, s>>>(b, sd.bpart, sd.bent, Linv, y, x, sd.partials, sd.arrive,
                                                     sd.done, sd.epoch, fail);
    return;
  }
  for (size_t lv = 0; lv + 1 < blevel.size(); ++lv) {
    const int n = blevel[lv + 1] - blevel[lv];
    if (n > 0) k_back<<<n, kBackThreads, 0, s>>>(b, sd.bpart + blevel[lv], sd.bent, Linv, y, x, sd.partials, sd.arrive);
  }
}

void launch_small_solve(const TileDev& b, const SmallMap& m, const double* r, double* x, int* fail, hipStream_t s) {
  if (b.NT <= 0 || b.NT > kSmallNT) return;   // the host checks the size (solver.cpp)
  k_small_solve<<<1, kSW * 64, 0, s>>>(b, m, r, x, fail);
}

}  // namespace dynohip
