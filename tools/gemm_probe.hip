// 64x64x64 FP64 GEMM probe on LDS operands: MFMA f64 16x16x4 vs VALU 4x4 tiles.
#include "../dynosam_amd/csrc/band.hip"
#include <cstdio>
using namespace dynohip;

__device__ void valu_abt(const double* As, const double* Bs, int tid, double acc[4][4]) {
  const int r0 = (tid >> 4) * 4, c0 = (tid & 15) * 4;
  for (int u = 0; u < 4; ++u) for (int w = 0; w < 4; ++w) acc[u][w] = 0.0;
#pragma unroll 4
  for (int m = 0; m < T; ++m) {
    double a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) { a[u] = As[(r0 + u) * LD + m]; b[u] = Bs[(c0 + u) * LD + m]; }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int w = 0; w < 4; ++w) acc[u][w] += a[u] * b[w];
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void k_gemm(const double* src, double* out, long long* cyc, int reps) {
  __shared__ double As[T * LD], Bs[T * LD];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  load_tile_lds(src, As, tid, 256);
  load_tile_lds(src + 4096, Bs, tid, 256);
  __syncthreads();
  double s = 0;
  long long t0 = clock64();
  for (int it = 0; it < reps; ++it) {
    if (MODE == 0) {
      v4d acc[2][2];
      mfma_abt(As, Bs, w, l, acc);
      for (int a = 0; a < 2; ++a) for (int b = 0; b < 2; ++b) for (int r = 0; r < 4; ++r) s += acc[a][b][r];
    } else {
      double acc[4][4];
      valu_abt(As, Bs, tid, acc);
      for (int a = 0; a < 4; ++a) for (int b = 0; b < 4; ++b) s += acc[a][b];
    }
  }
  long long t1 = clock64();
  out[blockIdx.x * 256 + tid] = s;
  if (tid == 0) cyc[blockIdx.x] = (t1 - t0) / reps;
}

int main() {
  double *src, *out; long long* cyc;
  hipMalloc(&src, 8192 * 8); hipMalloc(&out, 256 * 1024 * 8); hipMalloc(&cyc, 1024 * 8);
  hipMemset(src, 0, 8192 * 8);
  long long c;
  for (int blocks : {1, 256}) {
    k_gemm<0><<<blocks, 256>>>(src, out, cyc, 50); hipDeviceSynchronize();
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("blocks=%d MFMA f64 64^3: %lld cycles per GEMM\n", blocks, c);
    k_gemm<1><<<blocks, 256>>>(src, out, cyc, 50); hipDeviceSynchronize();
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("blocks=%d VALU f64 64^3: %lld cycles per GEMM\n", blocks, c);
  }
  return 0;
}
