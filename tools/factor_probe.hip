// Development probe: the 64x64 diagonal-tile factorisation + inverse of
// tilechol.hip (factor_tile_blk: 16x16 in-wave blocks), timed and checked
// against a host Cholesky inverse.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/factor_probe.hip -o tools/factor_probe
#include "../dynosam_amd/csrc/tilechol.hip"

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

using namespace dynohip;

// ablation: the blocked factor without the inverse (X) work
__device__ bool factor_tile_noX(v4d (&accA)[4], int w, int l, double* xch) {
  bool ok = true;
#pragma unroll
  for (int KB = 0; KB < 4; ++KB) {
    double* xb = xch + (KB & 1) * 4 * 256;
    if (w == KB) {
      v4d W = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int r = 0; r < 4; ++r) W[r] = ((l >> 4) + 4 * r == (l & 15)) ? 1.0 : 0.0;
      factor16_wave(accA[KB], W, l, ok);
#pragma unroll
      for (int TJ = 0; TJ < 4; ++TJ) {
        v4d z = v4d{0.0, 0.0, 0.0, 0.0};
        if (TJ > KB) {
          accA[TJ] = mfma_tn(W, accA[TJ], z, false);
#pragma unroll
          for (int r = 0; r < 4; ++r) xb[TJ * 256 + r * 64 + l] = accA[TJ][r];
        }
      }
    }
    __syncthreads();
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
    }
  }
  return ok;
}


template <int V>
__global__ __launch_bounds__(256) void k_fact(const double* A, double* X, long long* cyc, int* okout) {
  __shared__ double buf[2 * T * 4 + 2 * 4 * T + 2 * 4 * 256];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  v4d accA[4], accX[4];
  for (int TJ = 0; TJ < 4; ++TJ)
    for (int r = 0; r < 4; ++r) {
      const int row = ACC_ROW(w, l, r), col = ACC_COL(TJ, l);
      accA[TJ][r] = row >= col ? A[row * T + col] : A[col * T + row];
      accX[TJ][r] = row == col ? 1.0 : 0.0;
    }
  __syncthreads();
  const long long t0 = clock64();
  bool ok;
  if (V == 1) ok = factor_tile_blk(accA, accX, w, l, buf);
  else ok = factor_tile_noX(accA, w, l, buf);
  __syncthreads();
  const long long t1 = clock64();
  for (int TJ = 0; TJ < 4; ++TJ)
    for (int r = 0; r < 4; ++r) X[ACC_ROW(w, l, r) * T + ACC_COL(TJ, l)] = accX[TJ][r];
  if (tid == 0) { cyc[blockIdx.x] = t1 - t0; okout[0] = ok; }
}

int main() {
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
  // host: L = chol(A), Xref = L^-1
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
  for (int V = 1; V < 3; ++V) {
    auto launch = [&](int n) { if (V == 1) k_fact<1><<<n, 256>>>(dA, dX, cyc, ok); else k_fact<2><<<n, 256>>>(dA, dX, cyc, ok); };
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
    printf("variant %d: ok=%d  max|X-Xref|/max|Xref| = %.3e  clock64 ticks = %lld  launch = %.2f us\n", V, okh,
           err / mx, c, ms * 1e3 / 200);
  }
  return 0;
}
