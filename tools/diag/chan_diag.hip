// chan_diag.hip -- chan_tile_kernel on a small fp32 signal against a CPU
// reference; prints the mismatch pattern by (wave, block, channel, frame).
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/diag/chan_diag tools/diag/chan_diag.hip \
//          digital_signal_processsing_amd/csrc/mavg_common.hip -Ldigital_signal_processsing_amd/lib -lmavg
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
#include "../../digital_signal_processsing_amd/csrc/mavg_launch.hpp"
using namespace mavg;
template <int C, int Q, int WG>
int run(int k, long long nframes) {
  const long long n = nframes * C;
  std::vector<float> hx(n), hy(n);
  for (long long i = 0; i < n; ++i) hx[i] = (float)((i * 2654435761u) % 1000) / 100.0f;
  float *x, *y;
  hipMalloc(&x, n * 4);
  hipMalloc(&y, n * 4);
  hipMemcpy(x, hx.data(), n * 4, hipMemcpyHostToDevice);
  hipMemset(y, 0, n * 4);
  const Sig sg{x, y, nullptr, nframes};
  constexpr int kNtS = kNtSplit | kNtHalo | kNtStore;
  int rc = launch_chan_tile<float, double, C, Q, WG, kNtS>(sg, k, 0);
  hipDeviceSynchronize();
  hipMemcpy(hy.data(), y, n * 4, hipMemcpyDeviceToHost);
  constexpr int NB = 64 / C, WF = NB * Q, TF = (WG / 64) * WF;
  long long bad = 0;
  std::vector<long long> byw(WG / 64), byb(NB), byc(C), byi(Q);
  for (int c = 0; c < C; ++c) {
    double s = 0;
    for (long long f = 0; f < nframes; ++f) {
      s += hx[f * C + c];
      if (f >= k) s -= hx[(f - k) * C + c];
      const double r = s / k;
      const double g = hy[f * C + c];
      if (std::fabs(g - r) > 1e-4 * std::fabs(r) + 1e-5) {
        if (bad < 10) printf("bad f=%lld c=%d got %g want %g\n", f, c, g, r);
        ++bad;
        const int ft = (int)(f % TF);
        byw[ft / WF]++;
        byb[(ft % WF) / Q]++;
        byc[c]++;
        byi[ft % Q]++;
      }
    }
  }
  printf("C=%d Q=%d WG=%d k=%d rc=%d bad=%lld of %lld\n by wave:", C, Q, WG, k, rc, bad, n);
  for (auto v : byw) printf(" %lld", v);
  printf("\n by block:");
  for (auto v : byb) printf(" %lld", v);
  printf("\n by channel:");
  for (auto v : byc) printf(" %lld", v);
  printf("\n by frame in block:");
  for (auto v : byi) printf(" %lld", v);
  printf("\n");
  hipFree(x);
  hipFree(y);
  return 0;
}
int main() {
  run<8, 16, 256>(7, 1024 * 40 + 3);
  run<8, 16, 256>(100, 1024 * 40);
  run<4, 16, 256>(7, 1024 * 40);
  return 0;
}
