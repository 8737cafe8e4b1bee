// Development probe: cost per pivot of the in-wave 16x16 factorisation and
// of its ingredients (cycles per call, one wave).
#include "../dynosam_amd/csrc/tilechol.hip"
#include <cstdio>
using namespace dynohip;

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
  double acc = 0.0;
  const long long t0 = clock64();
  for (int it = 0; it < 8; ++it) {
    if (V == 0) factor16_wave(B, W, l, ok);
    if (V == 1) {  // rsqrt chain only
#pragma unroll
      for (int p = 0; p < 16; ++p) B[0] = rsqrt_nr(B[0] + 1.0);
    }
    if (V == 2) {  // bpermute chain only
#pragma unroll
      for (int p = 0; p < 16; ++p) B[0] = pull_lane(B[0], (l + p) & 63) + 1.0;
    }
    if (V == 3) {  // readlane chain only
#pragma unroll
      for (int p = 0; p < 16; ++p) B[0] = read_lane(B[0], p) + 1.0;
    }
    if (V == 4) {  // dpp chain only
#pragma unroll
      for (int p = 0; p < 16; ++p) B[0] = bcast_row_lane(B[0], p) + 1.0;
    }
    if (V == 5) {  // fma chain only
#pragma unroll
      for (int p = 0; p < 16; ++p) B[0] = B[0] * 0.999 + 1e-3;
    }
    acc += B[0] + W[1];
  }
  const long long t1 = clock64();
  out[l] = acc + ok;
  if (l == 0) cyc[V] = (t1 - t0) / (8 * 16);
}

int main() {
  double* out; long long* cyc;
  hipMalloc(&out, 64 * 8); hipMalloc(&cyc, 16 * 8);
  k_piv<0><<<1, 64>>>(out, cyc); k_piv<1><<<1, 64>>>(out, cyc); k_piv<2><<<1, 64>>>(out, cyc);
  k_piv<3><<<1, 64>>>(out, cyc); k_piv<4><<<1, 64>>>(out, cyc); k_piv<5><<<1, 64>>>(out, cyc);
  hipDeviceSynchronize();
  long long h[16]; hipMemcpy(h, cyc, 16 * 8, hipMemcpyDeviceToHost);
  const char* names[] = {"factor16 pivot", "rsqrt_nr", "bpermute(f64)", "readlane(f64)", "dpp newbcast", "fma"};
  for (int v = 0; v < 6; ++v) printf("%-16s %lld cycles per step\n", names[v], h[v]);
  return 0;
}
