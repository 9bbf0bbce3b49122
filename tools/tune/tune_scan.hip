// tune_scan.hip -- interleaved A/B timing of scan_kernel variants against an
// HBM copy ceiling on one MI355X (cdna_hip_programming.md 5.4 rule 24: all
// variants in ONE process, interleaved rounds, median and min reported).
// Every scan variant's output is compared bit-for-bit with the first one.
//
// build: make -C tools/tune
// run:   tools/tune/tune_scan [log2n] [k] [rounds] [f32|i16] [burst] [filter] [channels (i16: 1|2)]
//        burst > 0: launches per event pair (mean); burst < 0: -burst back-to-back launches with one
//        event pair each, as bench.py times them (the two orderings can rank tile shapes differently)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "../../digital_signal_processsing_amd/csrc/mavg_launch.hpp"

using namespace mavg;

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

// float4 streaming copy: the achievable-bandwidth reference for 4 B in + 4 B out
template <int NT, int UNR>
__global__ __launch_bounds__(256) void copy_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out,
                                                   long long n4) {
  const long long stride = (long long)gridDim.x * 256 * UNR;
  for (long long i = (long long)blockIdx.x * 256 * UNR + threadIdx.x; i < n4; i += stride) {
    u32x4 v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const long long j = i + u * 256;
      if (j < n4) v[u] = (NT & 2) ? __builtin_nontemporal_load(in + j) : in[j];
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const long long j = i + u * 256;
      if (j < n4) {
        if (NT & 1) __builtin_nontemporal_store(v[u], out + j);
        else out[j] = v[u];
      }
    }
  }
}

template <int NT>
__global__ __launch_bounds__(256) void flat_copy(const u32x4* __restrict__ in, u32x4* __restrict__ out, long long n4) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < n4) {
    u32x4 v = (NT & 2) ? __builtin_nontemporal_load(in + i) : in[i];
    if (NT & 1) __builtin_nontemporal_store(v, out + i);
    else out[i] = v;
  }
}

__global__ void count_diff(const uint32_t* a, const uint32_t* b, long long n, unsigned long long* cnt) {
  unsigned long long c = 0;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    c += a[i] != b[i];
  if (c) atomicAdd(cnt, c);
}

struct Variant {
  std::string name;
  bool is_scan;
  std::function<int(hipStream_t)> launch;
  std::vector<float> ms;
  unsigned long long mism = 0;
};

template <typename T, typename A>
void add_variants(std::vector<struct Variant>& vs, T* x, T* y, long long n, int k);

static int g_burst = 1;  // launches per timed sample (back-to-back, like bench.py's steps)
static int g_channels = 1;  // 2: int16 stereo variants (interleaved frames)
static Workspace g_ws;      // look-back scan workspace (64 MiB, allocated in run())
static std::string g_filter;  // "a|b": keep only variants whose name contains a or b

static bool keep(const std::string& name) {
  if (g_filter.empty()) return true;
  size_t st = 0;
  while (st <= g_filter.size()) {
    size_t e = g_filter.find('|', st);
    if (e == std::string::npos) e = g_filter.size();
    if (name.find(g_filter.substr(st, e - st)) != std::string::npos) return true;
    st = e + 1;
  }
  return false;
}

template <typename T, typename A>
int run(int lg, int k, int rounds) {
  const long long n = 1LL << lg;
  constexpr int ES = sizeof(T);
  T *x, *y, *yref;
  CK(hipMalloc(&x, n * ES));
  CK(hipMalloc(&y, n * ES));
  CK(hipMalloc(&yref, n * ES));
  unsigned long long* dcnt;
  CK(hipMalloc(&dcnt, 8));
  g_ws.bytes = 64u << 20;
  CK(hipMalloc(&g_ws.ptr, g_ws.bytes));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipLaunchKernelGGL(synth_kernel<T>, dim3(4096), dim3(256), 0, st, x, n, (uint64_t)0x5EED, 0);
  CK(hipStreamSynchronize(st));
  int cus = device_cu_count();
  printf("device CUs=%d n=2^%d k=%d rounds=%d dtype=%s y-x=%#llx\n", cus, lg, k, rounds, ES == 4 ? "f32" : "i16",
         (unsigned long long)((const char*)y - (const char*)x));

  std::vector<Variant> vs;
  const long long n4 = n * ES / 16;
  auto add_copy = [&](const char* nm, auto kern, int grid) {
    vs.push_back({nm, false, [=](hipStream_t s) {
                    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, s, (const u32x4*)x, (u32x4*)y, n4);
                    return 0;
                  }});
  };
  add_copy("copy gs g16384 u2 ntLS", copy_kernel<3, 2>, 16384);
  add_copy("copy flat u1 ntLS", flat_copy<3>, (int)(n4 / 256));

  add_variants<T, A>(vs, x, y, n, k);
  {
    std::vector<Variant> kept;
    for (auto& v : vs)
      if (keep(v.name)) kept.push_back(v);
    vs.swap(kept);
  }

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<hipEvent_t> ce(g_burst < 0 ? 2 * (-g_burst) : 0);
  for (auto& e : ce) CK(hipEventCreate(&e));
  // reference output + correctness of every scan variant
  bool have_ref = false;
  {  // drop variants the launcher refuses (e.g. LDS over budget for this k)
    std::vector<Variant> ok;
    for (auto& v : vs) {
      if (v.launch(st) != 0) printf("%s: launch refused, skipped\n", v.name.c_str());
      else ok.push_back(v);
    }
    vs.swap(ok);
    CK(hipStreamSynchronize(st));
  }
  for (auto& v : vs) {
    if (!v.is_scan) continue;
    if (v.launch(st) != 0) { printf("%s: launch failed\n", v.name.c_str()); return 1; }
    CK(hipStreamSynchronize(st));
    if (!have_ref) {
      CK(hipMemcpyAsync(yref, y, n * ES, hipMemcpyDeviceToDevice, st));
      have_ref = true;
    } else {
      CK(hipMemsetAsync(dcnt, 0, 8, st));
      hipLaunchKernelGGL(count_diff, dim3(2048), dim3(256), 0, st, (const uint32_t*)y, (const uint32_t*)yref,
                         n * ES / 4, dcnt);
      CK(hipMemcpyAsync(&v.mism, dcnt, 8, hipMemcpyDeviceToHost, st));
    }
    CK(hipStreamSynchronize(st));
    if (v.name.find("ahead") != std::string::npos && v.name.find("product") == std::string::npos) {
      LaunchPlan lp{};
      g_plan = &lp;
      v.launch(st);
      g_plan = nullptr;
      unsigned int stt[2] = {0, 0};
      CK(hipMemcpy(stt, static_cast<unsigned char*>(g_ws.ptr) + lp.ws_bytes - 16, 8, hipMemcpyDeviceToHost));
      printf("%s: recomputes = %u, waiting polls = %u\n", v.name.c_str(), stt[0], stt[1]);
    }
    if (v.name.find("onepass") != std::string::npos) {
      unsigned int fb = 0;
      CK(hipMemcpy(&fb, g_ws.ptr, 4, hipMemcpyDeviceToHost));
      printf("%s: record recomputes (fallbacks) = %u\n", v.name.c_str(), fb);
    }
    CK(hipMemsetAsync(y, 0xff, n * ES, st));
  }
  for (auto& v : vs) { v.launch(st); v.launch(st); }
  CK(hipStreamSynchronize(st));
  // the start of each round rotates, so every variant follows every other one
  // equally often (a fixed order measured the variant right after the copy
  // 1-3 % slow)
  for (int r = 0; r < rounds; ++r) {
    for (size_t j = 0; j < vs.size(); ++j) {
      auto& v = vs[(j + r) % vs.size()];
      if (g_burst < 0) {
        // bench.py's timing: -burst back-to-back launches, one event pair each
        for (int b = 0; b < -g_burst; ++b) {
          CK(hipEventRecord(ce[2 * b], st));
          v.launch(st);
          CK(hipEventRecord(ce[2 * b + 1], st));
        }
        CK(hipEventSynchronize(ce[2 * (-g_burst) - 1]));
        for (int b = 0; b < -g_burst; ++b) {
          float ms;
          CK(hipEventElapsedTime(&ms, ce[2 * b], ce[2 * b + 1]));
          v.ms.push_back(ms);
        }
        continue;
      }
      CK(hipEventRecord(e0, st));
      for (int b = 0; b < g_burst; ++b) v.launch(st);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms / g_burst);
    }
  }
  // frac8T from the median; bench.py reports the mean (mfrac8T), which a
  // variant with a few slow launches loses (int16 LDS-DMA tiles did)
  printf("%-28s %9s %9s %9s %9s %s %9s\n", "variant", "med_ms", "min_ms", "GB/s", "frac8T", "mismatch", "mfrac8T");
  for (auto& v : vs) {
    std::vector<float> m = v.ms;
    std::sort(m.begin(), m.end());
    const float med = m[m.size() / 2], mn = m[0];
    double mean = 0;
    for (float t : m) mean += t;
    mean /= (double)m.size();
    const double gbs = 2.0 * ES * n / (med * 1e-3) / 1e9;
    const double mgbs = 2.0 * ES * n / (mean * 1e-3) / 1e9;
    printf("%-28s %9.4f %9.4f %9.1f %9.4f %llu %9.4f\n", v.name.c_str(), med, mn, gbs, gbs / 8000.0, v.mism,
           mgbs / 8000.0);
  }
  CK(hipFree(x));
  CK(hipFree(y));
  CK(hipFree(yref));
  return 0;
}

// variant lists (macros expand to launches of the library's launch helpers)
template <>
void add_variants<float, double>(std::vector<Variant>& vs, float* x, float* y, long long n, int k) {
#define TILE(U, NT, RM)                                                                                  \
  vs.push_back({"tile U" #U " NT" #NT " remap" #RM, true, [=](hipStream_t s) {                             \
                  return launch_tile_scan<float, double, 1, 4, U, false, NT>(Sig{x, y, nullptr, n}, k, s, RM);   \
                }});
#define DIRECT(U, WG)                                                                                   \
  vs.push_back({"direct U" #U " wg" #WG, true, [=](hipStream_t s) {                                        \
                  return launch_direct<float, double, 1, 4, U, WG>(Sig{x, y, nullptr, n}, k, s, 1);             \
                }});
#define TILEW(U, WG)                                                                                    \
  vs.push_back({"tile U" #U " wg" #WG, true, [=](hipStream_t s) {                                         \
                  return launch_tile_scan<float, double, 1, 4, U, false, 0, WG>(Sig{x, y, nullptr, n}, k, s, 1); \
                }});
#define TILEM(U, M)                                                                                     \
  vs.push_back({"tile U" #U " remap" #M, true, [=](hipStream_t s) {                                       \
                  return launch_tile_scan<float, double, 1, 4, U, false, 0>(Sig{x, y, nullptr, n}, k, s, M); \
                }});
#define DIRECTM(M)                                                                                      \
  vs.push_back({"direct U1 remap" #M, true, [=](hipStream_t s) {                                          \
                  return launch_direct<float, double, 1, 4, 1>(Sig{x, y, nullptr, n}, k, s, M);                 \
                }});
  vs.push_back({"hillis tile U2", true, [=](hipStream_t s) {
                  return launch_tile_scan<float, double, 1, 4, 2, true, 0>(Sig{x, y, nullptr, n}, k, s);
                }});
#define HTS(U, NT, WG)                                                                                  \
  vs.push_back({"hillisS U" #U " nt" #NT " wg" #WG, true, [=](hipStream_t s) {                              \
                  return launch_tile_scan<float, double, 1, 4, U, true, NT, WG>(Sig{x, y, nullptr, n}, k, s);     \
                }});
  HTS(2, 0, 256)
  HTS(2, 1, 256)
  HTS(2, 3, 256)
  HTS(2, 13, 256)
  HTS(1, 13, 256)
  HTS(2, 13, 512)
  HTS(4, 13, 256)
  HTS(4, 3, 256)
  HTS(4, 1, 256)
  HTS(8, 13, 256)
  HTS(8, 3, 256)
  HTS(4, 13, 512)
  HTS(2, 3, 512)
  HTS(2, 13, 1024)
  HTS(4, 13, 1024)
  vs.push_back({"hillis tile U1", true, [=](hipStream_t s) {
                  return launch_tile_scan<float, double, 1, 4, 1, true, 0>(Sig{x, y, nullptr, n}, k, s);
                }});
#define TILENR(U, NT)                                                                                   \
  vs.push_back({"tile U" #U " NT" #NT " noRC", true, [=](hipStream_t s) {                                 \
                  return launch_tile_scan<float, double, 1, 4, U, false, NT, 256, false>(Sig{x, y, nullptr, n}, k, s); \
                }});
  TILENR(2, 0)
  TILENR(4, 3)
  TILENR(8, 0)
#define TDMA(U, NT, WG, DMA)                                                                            \
  vs.push_back({"tdma U" #U " nt" #NT " wg" #WG " dma" #DMA, true, [=](hipStream_t s) {                   \
                  return launch_tile_scan<float, double, 1, 4, U, false, NT, WG, true, 0, DMA>(Sig{x, y, nullptr, n}, k, s, 64); \
                }});
  TDMA(2, 13, 256, false) TDMA(2, 13, 256, true) TDMA(2, 3, 256, false) TDMA(2, 3, 512, false) TDMA(2, 3, 512, true)
  TDMA(4, 13, 512, false) TDMA(4, 13, 512, true) TDMA(2, 13, 512, false) TDMA(2, 13, 512, true) TDMA(1, 13, 1024, true)
  TDMA(2, 13, 1024, true) TDMA(3, 13, 1024, true) TDMA(3, 13, 512, true)
#define TILEWG(U, WG)                                                                                   \
  vs.push_back({"tile U" #U " wg" #WG " rc", true, [=](hipStream_t s) {                                   \
                  return launch_tile_scan<float, double, 1, 4, U, false, 0, WG>(Sig{x, y, nullptr, n}, k, s, 64); \
                }});
#define TILEX(U, NT, WG, RC)                                                                            \
  vs.push_back({"tileX U" #U " nt" #NT " wg" #WG " rc" #RC, true, [=](hipStream_t s) {                    \
                  return launch_tile_scan<float, double, 1, 4, U, false, NT, WG, RC>(Sig{x, y, nullptr, n}, k, s, 64); \
                }});
  TILEX(2, 1, 256, false)
  TILEX(2, 0, 512, false)
  TILEX(2, 1, 512, true)
  TILEX(2, 0, 1024, true)
  TILEX(1, 0, 1024, true)
  TILEX(2, 0, 512, true)
  TILEX(2, 0, 256, true)
  TILEX(2, 0, 256, false)
  TILEX(4, 0, 256, false)
  TILEX(4, 3, 256, false)
  TILEX(4, 3, 256, true)
  TILEX(4, 1, 256, true)
  TILEX(2, 1, 256, true)
  TILEX(8, 3, 256, true)
  TILEX(4, 0, 128, true)
  TILEX(8, 0, 128, true)
  TILEX(4, 0, 128, false)
  TILEWG(8, 256)
  TILEWG(4, 256)
  TILEWG(4, 512)
  TILEWG(2, 1024)
  TILEWG(2, 256)
  TILEWG(2, 512)
  // clean grid for the dispatch rules (tools/tune/sweep_shapes.sh)
#define AH2(U, RC, DMA, D, W, NT)                                                                       \
  vs.push_back({"ahead U" #U " rc" #RC " dma" #DMA " D" #D " w" #W " nt" #NT, true, [=](hipStream_t s) { \
                  return launch_ahead_scan<float, double, 1, 4, U, NT, RC, DMA, W>(Sig{x, y, nullptr, n}, k, s, g_ws, D); \
                }});
  AH2(4, false, false, 1024, false, 1) AH2(4, false, false, 1024, false, 9) AH2(4, false, false, 512, false, 9)
  AH2(4, true, true, 512, true, 1) AH2(4, true, true, 512, true, 9) AH2(4, true, true, 1024, true, 9)
  AH2(4, false, true, 512, true, 9) AH2(4, false, true, 1024, true, 9) AH2(4, true, true, 768, true, 9)
#define TILES(U, NT, WG)                                                                                \
  vs.push_back({"tileS U" #U " nt" #NT " wg" #WG, true, [=](hipStream_t s) {                               \
                  return launch_tile_scan<float, double, 1, 4, U, false, NT, WG, true>(Sig{x, y, nullptr, n}, k, s, 64); \
                }});
  TILES(2, 0, 256)
  TILES(2, 1, 256)
  TILES(2, 4, 256)
  TILES(2, 5, 256)
  TILES(2, 12, 256)
  TILES(2, 13, 256)
  TILES(4, 0, 512)
  TILES(4, 4, 512)
  TILES(4, 5, 512)
  TILES(4, 13, 512)
  TILES(4, 13, 256)
  TILES(2, 3, 256)
  TILES(4, 3, 256)
  TILES(4, 1, 512)
  TILES(2, 0, 512)
  TILES(2, 1, 512)
  TILES(2, 5, 512)
  TILES(2, 13, 512)
  TILES(2, 0, 1024)
  TILES(2, 1, 1024)
  TILES(2, 5, 1024)
  TILES(2, 13, 1024)
  TILE(1, 0, 64)
  TILE(2, 0, 64)
  TILE(2, 1, 64)
  TILE(2, 2, 64)
  TILE(2, 3, 64)
  TILE(4, 0, 64)
  TILE(4, 3, 64)
  TILE(8, 0, 64)
  TILE(8, 3, 64)
  vs.push_back({"f32 product mavg_run", true, [=](hipStream_t s) {
                  return mavg_run(x, y, n, 1, k, MAVG_F32, MAVG_ALGO_AUTO, 0, nullptr, g_ws.ptr, g_ws.bytes, s);
                }});
  vs.push_back({"f32 disp", true, [=](hipStream_t s) {
                  return dispatch_scan_f<float, double, 1, 4, false>(Sig{x, y, nullptr, n}, k, 0, s, g_ws);
                }});
  TILEM(1, 1)
  TILEM(1, 64)
  TILEM(4, 1)
  TILEM(4, 64)
  TILEM(2, 1)
  TILEM(2, 4)
  TILEM(2, 16)
  TILEM(2, 64)
  TILEM(2, 256)
  TILEM(2, 1024)
  TILEM(8, 1)
  TILEM(8, 16)
  TILEM(8, 64)
  TILEM(8, 256)
#define DIRW(U, WG)                                                                                     \
  vs.push_back({"dirw U" #U " wg" #WG, true, [=](hipStream_t s) {                                         \
                  return launch_direct<float, double, 1, 4, U, WG>(Sig{x, y, nullptr, n}, k, s, 64);         \
                }});
  DIRW(1, 256) DIRW(2, 256) DIRW(4, 256) DIRW(1, 512) DIRW(2, 512) DIRW(1, 1024)
#define DIRNT(U, WG, NT)                                                                                \
  vs.push_back({"dirnt U" #U " wg" #WG " nt" #NT, true, [=](hipStream_t s) {                              \
                  return launch_direct<float, double, 1, 4, U, WG, NT>(Sig{x, y, nullptr, n}, k, s, kRemapGroup); \
                }});
  DIRNT(1, 256, 0) DIRNT(1, 256, 1) DIRNT(1, 256, 3) DIRNT(1, 256, 9) DIRNT(1, 256, 11)
  DIRNT(2, 256, 1) DIRNT(2, 256, 11) DIRNT(1, 512, 1) DIRNT(1, 512, 11)
  DIRECTM(1)
  DIRECTM(16)
  DIRECTM(64)
  DIRECTM(256)

}

template <>
void add_variants<int16_t, int32_t>(std::vector<Variant>& vs, int16_t* x, int16_t* y, long long n, int k) {
#define ITILE(U, M)                                                                                       \
  vs.push_back({"i16 tile U" #U " remap" #M, true, [=](hipStream_t s) {                                    \
                  return launch_tile_scan<int16_t, int32_t, 1, 8, U, false, 0>(Sig{x, y, nullptr, n}, k, s, M); \
                }});
#define ITILENT(U, NT)                                                                                    \
  vs.push_back({"i16 tile U" #U " NT" #NT, true, [=](hipStream_t s) {                                      \
                  return launch_tile_scan<int16_t, int32_t, 1, 8, U, false, NT>(Sig{x, y, nullptr, n}, k, s, 1); \
                }});
#define ITILENTR(U, NT, M)                                                                                \
  vs.push_back({"i16 tile U" #U " NT" #NT " remap" #M, true, [=](hipStream_t s) {                          \
                  return launch_tile_scan<int16_t, int32_t, 1, 8, U, false, NT>(Sig{x, y, nullptr, n}, k, s, M); \
                }});
#define IPROD()                                                                                           \
  vs.push_back({"i16 product mavg_run", true, [=](hipStream_t s) {                                        \
                  return mavg_run(x, y, n, 1, k, MAVG_I16, MAVG_ALGO_AUTO, 0, nullptr, g_ws.ptr, g_ws.bytes, s); \
                }});                                                                                                       \
  vs.push_back({"i16 disp", true, [=](hipStream_t s) {                                                    \
                  return dispatch_scan_f<int16_t, int32_t, 1, 8, false>(Sig{x, y, nullptr, n}, k, 0, s, g_ws);   \
                }});
#define IDIRECT(U)                                                                                        \
  vs.push_back({"i16 direct U" #U, true, [=](hipStream_t s) {                                              \
                  return launch_direct<int16_t, int32_t, 1, 8, U>(Sig{x, y, nullptr, n}, k, s, 1);               \
                }});
#define STILE(U, NT, M)                                                                                   \
  vs.push_back({"i16 stereo tile U" #U " NT" #NT " remap" #M, true, [=](hipStream_t s) {                   \
                  return launch_tile_scan<int16_t, int32_t, 2, 4, U, false, NT>(Sig{x, y, nullptr, n / 2}, k, s, M); \
                }});
  if (g_channels == 2) {
    vs.push_back({"i16 stereo product mavg_run", true, [=](hipStream_t s) {
                    return mavg_run(x, y, n, 2, k, MAVG_I16, MAVG_ALGO_AUTO, 0, nullptr, g_ws.ptr, g_ws.bytes, s);
                  }});
    // the product's dispatch compiled into this binary (separates the library's
    // code object and the C ABI's host path from the kernel itself)
    vs.push_back({"i16 stereo disp", true, [=](hipStream_t s) {
                    return dispatch_scan_f<int16_t, int32_t, 2, 4, false>(Sig{x, y, nullptr, n / 2}, k, 0, s, g_ws);
                  }});
#define SAH2(U, RC, DMA, D, W, NT)                                                                      \
  vs.push_back({"i16 stereo ahead U" #U " rc" #RC " dma" #DMA " D" #D " w" #W " nt" #NT, true, [=](hipStream_t s) {\
                  return launch_ahead_scan<int16_t, int32_t, 2, 4, U, NT, RC, DMA, W>(Sig{x, y, nullptr, n / 2}, k, s, g_ws, D); \
                }});
    SAH2(4, false, true, 768, false, 9) SAH2(4, false, true, 1024, false, 9)
#define SAHDV(D, W, DV)                                                                                 \
  vs.push_back({"i16 stereo ahead D" #D " w" #W " div" #DV, true, [=](hipStream_t s) {                   \
                  return launch_ahead_scan<int16_t, int32_t, 2, 4, 4, 9, false, true, W, DV>(Sig{x, y, nullptr, n / 2}, k, s, g_ws, D); \
                }});
    SAHDV(768, false, 1) SAHDV(1024, false, 1) SAHDV(512, false, 1) SAHDV(512, true, 1)
    if (k > 65535) {
    }
#define STILES(U, NT, WG)                                                                               \
  vs.push_back({"i16 stereo tileS U" #U " nt" #NT " wg" #WG, true, [=](hipStream_t s) {                   \
                  return launch_tile_scan<int16_t, int32_t, 2, 4, U, false, NT, WG, false>(Sig{x, y, nullptr, n / 2}, k, s, 64); \
                }});
#define STILEDV(U, NT, DV)                                                                              \
  vs.push_back({"i16 stereo tile U" #U " nt" #NT " div" #DV, true, [=](hipStream_t s) {                   \
                  return launch_tile_scan<int16_t, int32_t, 2, 4, U, false, NT, 256, false, DV>(Sig{x, y, nullptr, n / 2}, k, s, 64); \
                }});
    STILEDV(4, 3, 0) STILEDV(4, 3, 1) STILEDV(4, 13, 0) STILEDV(4, 13, 1)
#define STDMA(U, NT, DMA)                                                                               \
  vs.push_back({"i16 stereo tdma U" #U " nt" #NT " dma" #DMA, true, [=](hipStream_t s) {                  \
                  return launch_tile_scan<int16_t, int32_t, 2, 4, U, false, NT, 256, false, 1, DMA>(Sig{x, y, nullptr, n / 2}, k, s, 64); \
                }});
    STDMA(4, 3, false) STDMA(4, 3, true) STDMA(8, 13, false) STDMA(8, 13, true)
#define STDMW(U, NT, WG, DMA)                                                                           \
  vs.push_back({"i16 stereo tdmw U" #U " nt" #NT " wg" #WG " dma" #DMA, true, [=](hipStream_t s) {        \
                  return launch_tile_scan<int16_t, int32_t, 2, 4, U, false, NT, WG, false, 1, DMA>(Sig{x, y, nullptr, n / 2}, k, s, 64); \
                }});
    STDMW(2, 3, 256, false) STDMW(2, 3, 512, false) STDMW(2, 3, 512, true) STDMW(2, 13, 512, true) STDMW(4, 13, 512, true) STDMW(4, 3, 512, false)
    STILES(4, 0, 256)
    STILES(4, 3, 256)
    STILES(4, 4, 256)
    STILES(4, 5, 256)
    STILES(4, 13, 256)
    STILES(4, 0, 512)
    STILES(4, 5, 512)
    STILES(4, 13, 512)
    STILES(2, 0, 1024)
    STILES(2, 5, 1024)
    STILES(2, 13, 1024)
#define SHTS(U, NT, WG)                                                                                 \
  vs.push_back({"i16 stereo hillisS U" #U " nt" #NT " wg" #WG, true, [=](hipStream_t s) {                 \
                  return launch_tile_scan<int16_t, int32_t, 2, 4, U, true, NT, WG>(Sig{x, y, nullptr, n / 2}, k, s); \
                }});
    SHTS(4, 0, 256)
    SHTS(4, 3, 256)
    SHTS(4, 13, 256)
    SHTS(8, 3, 256)
    SHTS(8, 13, 256)
    SHTS(4, 13, 512)
#define STILEWG(U, WG, RC)                                                                              \
  vs.push_back({"i16 stereo tile U" #U " wg" #WG " rc" #RC, true, [=](hipStream_t s) {                    \
                  return launch_tile_scan<int16_t, int32_t, 2, 4, U, false, 0, WG, RC>(Sig{x, y, nullptr, n / 2}, k, s, 64); \
                }});
    STILEWG(4, 256, false)
    STILEWG(2, 512, false)
    STILEWG(4, 512, false)
    STILEWG(2, 1024, false)
    STILEWG(1, 1024, false)
    STILEWG(4, 512, true)
#define STILENR(U, NT)                                                                                  \
  vs.push_back({"i16 stereo tile U" #U " NT" #NT " noRC", true, [=](hipStream_t s) {                      \
                  return launch_tile_scan<int16_t, int32_t, 2, 4, U, false, NT, 256, false>(Sig{x, y, nullptr, n / 2}, k, s); \
                }});
    STILENR(4, 3)
    STILENR(4, 0)
    STILE(2, 0, 64)
    STILE(2, 3, 64)
    STILE(4, 0, 64)
    STILE(4, 3, 64)
    STILE(8, 0, 64)
    STILE(8, 3, 64)
    return;
  }
#define ITILEWG(U, WG, RC)                                                                              \
  vs.push_back({"i16 tile U" #U " wg" #WG " rc" #RC, true, [=](hipStream_t s) {                           \
                  return launch_tile_scan<int16_t, int32_t, 1, 8, U, false, 0, WG, RC>(Sig{x, y, nullptr, n}, k, s, 64); \
                }});
  ITILEWG(8, 256, false)
  ITILEWG(4, 256, false)
  ITILEWG(4, 512, false)
  ITILEWG(2, 512, false)
  ITILEWG(4, 512, true)
  ITILEWG(2, 1024, false)
  ITILEWG(1, 1024, false)
#define IAH2(U, RC, DMA, D, W, NT)                                                                      \
  vs.push_back({"i16 ahead U" #U " rc" #RC " dma" #DMA " D" #D " w" #W " nt" #NT, true, [=](hipStream_t s) { \
                  return launch_ahead_scan<int16_t, int32_t, 1, 8, U, NT, RC, DMA, W>(Sig{x, y, nullptr, n}, k, s, g_ws, D); \
                }});
  IAH2(4, false, true, 512, true, 9) IAH2(4, false, true, 1024, false, 9)
#define IAHDV(D, W, DV)                                                                                 \
  vs.push_back({"i16 ahead D" #D " w" #W " div" #DV, true, [=](hipStream_t s) {                          \
                  return launch_ahead_scan<int16_t, int32_t, 1, 8, 4, 9, false, true, W, DV>(Sig{x, y, nullptr, n}, k, s, g_ws, D); \
                }});
  IAHDV(512, true, 1) IAHDV(1024, false, 1) IAHDV(768, false, 1)
  // 8-B units (F=4): x[n-k] unit-aligned when k = 4 mod 8 (e.g. 44100), register-staged
#define IAH4(U, D, W, DV)                                                                               \
  vs.push_back({"i16 ahead8B U" #U " D" #D " w" #W " div" #DV, true, [=](hipStream_t s) {                  \
                  return launch_ahead_scan<int16_t, int32_t, 1, 4, U, 9, false, false, W, DV>(Sig{x, y, nullptr, n}, k, s, g_ws, D); \
                }});
  IAH4(8, 512, true, 0) IAH4(8, 1024, false, 0) IAH4(4, 512, true, 0) IAH4(8, 512, true, 1)
  // tiny windows: AUTO's tile shape (halo <= 256 B: U2 nt3 x 256, magic division) vs the direct kernel
  vs.push_back({"i16 autotile U2 nt3", true, [=](hipStream_t s) {
                  return launch_tile_scan<int16_t, int32_t, 1, 8, 2, false, 3, 256, false>(Sig{x, y, nullptr, n}, k, s);
                }});
#define IDIRNT(U, NT)                                                                                   \
  vs.push_back({"i16 dirnt U" #U " nt" #NT, true, [=](hipStream_t s) {                                    \
                  return launch_direct<int16_t, int32_t, 1, 8, U, 256, NT>(Sig{x, y, nullptr, n}, k, s, kRemapGroup); \
                }});
  IDIRNT(2, 11) IDIRNT(1, 11) IDIRNT(1, 0)
  if (k > 65535) {
  }
#define ITILES(U, NT, WG)                                                                               \
  vs.push_back({"i16 tileS U" #U " nt" #NT " wg" #WG, true, [=](hipStream_t s) {                          \
                  return launch_tile_scan<int16_t, int32_t, 1, 8, U, false, NT, WG, false>(Sig{x, y, nullptr, n}, k, s, 64); \
                }});
#define ITILEDV(U, NT, DV)                                                                              \
  vs.push_back({"i16 tile U" #U " nt" #NT " div" #DV, true, [=](hipStream_t s) {                          \
                  return launch_tile_scan<int16_t, int32_t, 1, 8, U, false, NT, 256, false, DV>(Sig{x, y, nullptr, n}, k, s, 64); \
                }});
  ITILEDV(4, 3, 0) ITILEDV(4, 3, 1)
#define ITDMA(U, NT, DMA)                                                                               \
  vs.push_back({"i16 tdma U" #U " nt" #NT " dma" #DMA, true, [=](hipStream_t s) {                         \
                  return launch_tile_scan<int16_t, int32_t, 1, 8, U, false, NT, 256, false, 1, DMA>(Sig{x, y, nullptr, n}, k, s, 64); \
                }});
  ITDMA(4, 3, false) ITDMA(4, 3, true) ITDMA(8, 13, false) ITDMA(8, 13, true) ITDMA(4, 13, true)
#define ITDMW(U, NT, WG, DMA)                                                                           \
  vs.push_back({"i16 tdmw U" #U " nt" #NT " wg" #WG " dma" #DMA, true, [=](hipStream_t s) {               \
                  return launch_tile_scan<int16_t, int32_t, 1, 8, U, false, NT, WG, false, 1, DMA>(Sig{x, y, nullptr, n}, k, s, 64); \
                }});
  ITDMW(2, 3, 256, false) ITDMW(2, 3, 512, false) ITDMW(2, 3, 512, true) ITDMW(2, 13, 512, true) ITDMW(4, 13, 512, true) ITDMW(4, 3, 512, false)
  ITILES(4, 0, 256)
  ITILES(4, 3, 256)
  ITILES(4, 4, 256)
  ITILES(4, 5, 256)
  ITILES(4, 13, 256)
  ITILES(4, 0, 512)
  ITILES(4, 5, 512)
  ITILES(4, 13, 512)
  ITILES(2, 0, 1024)
  ITILES(2, 5, 1024)
  ITILES(2, 13, 1024)
#define IHTS(U, NT, WG)                                                                                 \
  vs.push_back({"i16 hillisS U" #U " nt" #NT " wg" #WG, true, [=](hipStream_t s) {                        \
                  return launch_tile_scan<int16_t, int32_t, 1, 8, U, true, NT, WG>(Sig{x, y, nullptr, n}, k, s); \
                }});
  IHTS(4, 0, 256)
  IHTS(4, 3, 256)
  IHTS(4, 13, 256)
  IHTS(8, 3, 256)
  IHTS(8, 13, 256)
  IHTS(4, 13, 512)
#define ITILENR(U, NT)                                                                                  \
  vs.push_back({"i16 tile U" #U " NT" #NT " noRC", true, [=](hipStream_t s) {                             \
                  return launch_tile_scan<int16_t, int32_t, 1, 8, U, false, NT, 256, false>(Sig{x, y, nullptr, n}, k, s); \
                }});
  ITILENR(4, 3)
  ITILENR(8, 0)
  ITILENTR(2, 0, 64)
  ITILENTR(2, 3, 64)
  ITILENTR(4, 0, 64)
  ITILENTR(4, 3, 64)
  ITILENTR(8, 0, 64)
  ITILENTR(8, 3, 64)
  IPROD()
  if (k <= 64) {
    IDIRECT(1)
    IDIRECT(2)
  }
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 30;
  const int k = argc > 2 ? atoi(argv[2]) : 1024;
  const int rounds = argc > 3 ? atoi(argv[3]) : 10;
  const std::string dt = argc > 4 ? argv[4] : "f32";
  g_burst = argc > 5 ? atoi(argv[5]) : 1;
  g_filter = argc > 6 ? argv[6] : "";
  g_channels = argc > 7 ? atoi(argv[7]) : 1;
  printf("burst=%d (launches per timed sample)\n", g_burst);
  return dt == "i16" ? run<int16_t, int32_t>(lg, k, rounds) : run<float, double>(lg, k, rounds);
}
