// Standalone timing of the band kernels (development tool): random SPD band,
// NT column tiles with D sub-diagonal tiles; times k_panel / k_update /
// k_band_back with HIP events; checks the solve residual on the host.
#include "../dynosam_amd/csrc/band.hip"

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

using namespace dynohip;

int main(int argc, char** argv) {
  const int NT = argc > 1 ? atoi(argv[1]) : 75;
  const int D = argc > 2 ? atoi(argv[2]) : 4;
  const int reps = argc > 3 ? atoi(argv[3]) : 5;
  const int n = NT * T;
  std::vector<int32_t> hD(NT), hc(NT);
  std::vector<int64_t> hoff(NT);
  int64_t off = 0;
  for (int j = 0; j < NT; ++j) {
    hD[j] = std::min(D, NT - 1 - j);
    hoff[j] = off;
    off += (int64_t)(hD[j] + 1) * T * T;
  }
  for (int i = 0; i < NT; ++i) hc[i] = std::max(0, i - D);
  // random banded SPD: A = B B^T + n I restricted to the band (diagonally dominant)
  std::mt19937_64 rng(1);
  std::uniform_real_distribution<double> U(-1, 1);
  std::vector<double> band(off, 0.0);
  auto at = [&](int r, int c) -> double& {
    int i = r / T, j = c / T;
    return band[hoff[j] + (int64_t)(i - j) * T * T + (r % T) * T + (c % T)];
  };
  const int bw = (D + 1) * T - 1;
  for (int r = 0; r < n; ++r)
    for (int c = std::max(0, (r / T - D) * T); c <= r; ++c) at(r, c) = (r == c) ? 2.0 * bw : U(rng);
  std::vector<double> g(n);
  for (auto& v : g) v = U(rng);
  double *dband, *dband0, *dlinv, *dr, *dy, *dx;
  int* dfail;
  int64_t* doff;
  int32_t *dD, *dc;
  hipMalloc(&dband, off * 8); hipMalloc(&dband0, off * 8);
  hipMalloc(&dlinv, (int64_t)NT * T * T * 8); hipMalloc(&dr, n * 8); hipMalloc(&dy, n * 8); hipMalloc(&dx, n * 8);
  hipMalloc(&dfail, 4); hipMalloc(&doff, NT * 8); hipMalloc(&dD, NT * 4); hipMalloc(&dc, NT * 4);
  hipMemcpy(dband0, band.data(), off * 8, hipMemcpyHostToDevice);
  hipMemcpy(doff, hoff.data(), NT * 8, hipMemcpyHostToDevice);
  hipMemcpy(dD, hD.data(), NT * 4, hipMemcpyHostToDevice);
  hipMemcpy(dc, hc.data(), NT * 4, hipMemcpyHostToDevice);
  BandDev b;
  b.NT = NT; b.n_red = n; b.band = dband; b.off = doff; b.D = dD; b.cmin = dc;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < reps; ++rep) {
    hipMemcpy(dband, dband0, off * 8, hipMemcpyDeviceToDevice);
    hipMemcpy(dr, g.data(), n * 8, hipMemcpyHostToDevice);
    hipMemset(dfail, 0, 4);
    hipDeviceSynchronize();
    hipEventRecord(e0, 0);
    launch_band_cholesky_solve(b, hD.data(), dlinv, dr, dy, dx, dfail, 0);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    best = std::min(best, ms);
  }
  std::vector<double> x(n);
  int fail = 0;
  hipMemcpy(x.data(), dx, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(&fail, dfail, 4, hipMemcpyDeviceToHost);
  // residual A x - g using the symmetric band
  double rn = 0, gn = 0;
  for (int r = 0; r < n; ++r) {
    double s = 0;
    for (int c = std::max(0, (r / T - D) * T); c <= std::min(n - 1, (r / T + D) * T + T - 1); ++c) {
      double a = c <= r ? band[hoff[c / T] + (int64_t)(r / T - c / T) * T * T + (r % T) * T + (c % T)]
                        : band[hoff[r / T] + (int64_t)(c / T - r / T) * T * T + (c % T) * T + (r % T)];
      if (c / T > r / T + D || r / T > c / T + D) a = 0;
      s += a * x[c];
    }
    rn += (s - g[r]) * (s - g[r]);
    gn += g[r] * g[r];
  }
  printf("NT=%d D=%d best %.3f ms  per-step %.2f us  fail=%d  rel-residual %.3e\n", NT, D, best, 1e3 * best / NT, fail,
         sqrt(rn / gn));
  return 0;
}
