// mavg_launch.hpp -- host-side launch helpers shared by the libmavg
// translation units (one TU per kernel family so the build parallelises).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "../../include/mavg.h"
#include "mavg_kernels.hpp"

namespace mavg {

constexpr int kMaxChannels = 8;
// tile -> XCD mapping of the flat-tile kernels: runs of 64 consecutive tiles
// per XCD, the 8 XCDs' runs adjacent (remap_tile in mavg_kernels.hpp)
constexpr int kRemapGroup = 64;
constexpr size_t kLdsBudget = 64 * 1024;  // per workgroup; keeps >= 2 workgroups per CU
// A 1024-thread workgroup may take 80 KiB: two of them still fill a CU's 32
// wave slots within its 160 KiB of LDS.
constexpr size_t lds_budget(int wg) { return wg >= 1024 ? 80 * 1024 : kLdsBudget; }

int device_cu_count();
OutParams make_out_params(int k);
constexpr int kMaxDevices = 64;  // per-device caches (CU count, dynamic-LDS limits)

// Raise one kernel's dynamic-LDS limit on the CURRENT device, once per
// (kernel, device): hipFuncSetAttribute acts on the current device, so a
// process that drives several devices must set it on each before it launches
// the kernel there (the 1024-thread tile takes 80 KiB).  Keyed on
// hipGetDevice; racing first calls both set it (idempotent).
template <auto Kernel>
int raise_dyn_lds_limit(int bytes) {
  static std::atomic<int> set_on[kMaxDevices];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return MAVG_ERR_HIP;
  const bool cached = dev >= 0 && dev < kMaxDevices;
  if (cached && set_on[dev].load(std::memory_order_acquire) == bytes) return MAVG_OK;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(Kernel), hipFuncAttributeMaxDynamicSharedMemorySize, bytes) !=
      hipSuccess)
    return MAVG_ERR_HIP;
  if (cached) set_on[dev].store(bytes, std::memory_order_release);
  return MAVG_OK;
}

// Dry-run support for mavg_plan(): when g_plan is set (thread-local), the
// launchers describe the launch they would make instead of making it.
struct LaunchPlan {
  char text[256];  // the longest plan (look-ahead with runs) is ~170 characters
  size_t ws_bytes;  // device workspace the launch needs (mavg_workspace_bytes)
};
extern thread_local LaunchPlan* g_plan;

template <typename T> constexpr const char* type_name();
template <> constexpr const char* type_name<float>() { return "f32"; }
template <> constexpr const char* type_name<int16_t>() { return "i16"; }
template <> constexpr const char* type_name<double>() { return "f64"; }
template <> constexpr const char* type_name<int32_t>() { return "i32"; }
template <> constexpr const char* type_name<int64_t>() { return "i64"; }

// One launch's view of the signal: caller-owned device pointers, the frame
// count, and two properties of a view the kernels must respect:
//   pre  frames in front of `in` that are readable signal: the body launch
//        after a peeled misaligned head (mavg_api.hip); `hist` then holds the
//        frames before those (load_elem)
//   eio  the pointers are only element-aligned: a frame-unit (F = 1) launch
//        moves multi-element frames as element accesses (UnitIO::gload)
struct Sig {
  const void* in;
  void* out;
  const void* hist;
  long long nframes;
  int pre = 0;
  int eio = 0;
};

// Workgroup size a non-zero reference block size (argv; a multiple of 32 in
// [32, 1024]) maps to: the next power of two, at least one wave64.
constexpr int block_wg(int block) {
  int wg = 64;
  while (wg < block && wg < 1024) wg <<= 1;
  return wg;
}

// family entry points (defined in mavg_scan_*.hip / mavg_direct.hip)
// Workspace: the look-ahead scan needs its record granules (ahead_granule_bytes)
// in caller-owned device memory (zeroed on the stream before each launch);
// every other launch needs none.
struct Workspace {
  void* ptr = nullptr;
  size_t bytes = 0;
};
// block: the reference's block size (0 = the tuned geometry)
int scan_f32(int C, bool vec, bool hs, const Sig& sg, int k, int block, hipStream_t st, Workspace ws);
int scan_i16(int C, bool vec, bool hs, const Sig& sg, int k, int block, hipStream_t st, Workspace ws);
int scan_i16_wide(int C, bool vec, bool hs, const Sig& sg, int k, int block, hipStream_t st, Workspace ws);
int direct_any(int dtype, bool wide, int C, int width, const Sig& sg, int k, int block, hipStream_t st);
int naive_any(int dtype, bool wide, const Sig& sg, int C, int k, int block, hipStream_t st);

// flat-tile scan: one workgroup per tile, carry rebuilt from the k-frame halo
// DV: the int16 output division of the tile scan -- the magic multiply, which
// measured faster than the fp64 product here (int16 stereo k=1024: 0.779 vs
// 0.763 of peak, mono equal; the look-ahead scan measured the other way,
// tools/tune/tune_scan.hip "div" variants)
template <typename T, typename A, int C, int F, int U, bool HS, int NT = kNtLoad | kNtStore, int WG = kWG,
          bool RC = true, int DV = (sizeof(T) == 2 ? 1 : 0), bool DMA = false>
int launch_tile_scan(const Sig& sg, int k, hipStream_t st, int xcd_remap = kRemapGroup) {
  constexpr int TF = WG * F * U;
  constexpr int NSEG = U * (WG / 64);
  constexpr int VE = F * C;
  const long long nframes = sg.nframes;
  TileParams p{};
  p.in = sg.in;
  p.out = sg.out;
  p.hist = sg.hist;
  p.nframes = nframes;
  p.pre = sg.pre;
  p.eio = sg.eio;
  p.k = k;
  p.o = make_out_params(k);
  p.halo_units = (k + F - 1) / F;
  p.xk_off = (int)((VE - ((long long)k * C) % VE) % VE);
  p.xcd_remap = xcd_remap;
  p.ntiles = (nframes + TF - 1) / TF;
  const size_t stage = (((size_t)(p.halo_units + U * WG + 1) * VE * sizeof(T)) + 15) & ~(size_t)15;
  const size_t lds = stage + (size_t)(NSEG + WG / 64) * C * sizeof(A);
  if (lds > lds_budget(WG)) return MAVG_ERR_UNSUPPORTED;
  if (p.ntiles > 0x7fffffffLL) return MAVG_ERR_UNSUPPORTED;
  if (g_plan) {
    snprintf(g_plan->text, sizeof(g_plan->text),
             "tile_scan<%s,acc=%s,C=%d,F=%d,U=%d,%s,nt=%d,rc=%d,dv=%d,dma=%d> grid=%lld block=%d lds=%zu "
             "tile_frames=%d remap=%d",
             type_name<T>(), type_name<A>(), C, F, U, HS ? "hillis" : "blelloch", NT, (int)RC, DV, (int)DMA,
             p.ntiles, WG, lds, TF, xcd_remap);
    return MAVG_OK;
  }
  if (lds > 64 * 1024) {  // beyond the default dynamic-LDS limit: raise it on this device
    const int st = raise_dyn_lds_limit<&tile_scan_kernel<T, A, C, F, U, HS, NT, WG, RC, DV, DMA>>((int)lds_budget(WG));
    if (st != MAVG_OK) return st;
  }
  hipLaunchKernelGGL((tile_scan_kernel<T, A, C, F, U, HS, NT, WG, RC, DV, DMA>), dim3((unsigned)p.ntiles), dim3(WG), lds, st,
                     p);
  return hipGetLastError() == hipSuccess ? MAVG_OK : MAVG_ERR_HIP;
}

// wide-frame tile scan (mavg_wide.hpp): lanes own chunks of P consecutive
// frames (64 or 128 B) of a multi-channel signal; 16-B-aligned views only
// (the host's vector path), halo + tile staged in a swizzled LDS stage.
template <typename T, typename A, int C, int P, int U, int WG, int NT, int DV = 0>
int launch_wide_tile(const Sig& sg, int k, hipStream_t st, int xcd_remap = kRemapGroup) {
  constexpr int EPG = 16 / (int)sizeof(T);
  constexpr int G = P * C / EPG;
  constexpr int TF = WG * P * U;
  constexpr int TG = WG * U * G;
  constexpr int NSEG = U * (WG / 64);
  const long long nframes = sg.nframes;
  const long long hg = ((long long)k * C + EPG - 1) / EPG;  // granules covering the k-frame halo
  const long long Hg = (hg + 15) / 16 * 16;                // whole 256-B LDS rows
  const size_t lds = (size_t)(Hg + TG) * 16 + (size_t)(NSEG + WG / 64) * C * sizeof(A);
  if (lds > 80 * 1024) return MAVG_ERR_UNSUPPORTED;  // two workgroups per CU at the longest halos
  const long long ntiles = (nframes + TF - 1) / TF;
  if (ntiles > 0x7fffffffLL) return MAVG_ERR_UNSUPPORTED;
  if (g_plan) {
    snprintf(g_plan->text, sizeof(g_plan->text),
             "wide_tile<%s,acc=%s,C=%d,P=%d,U=%d,nt=%d,dv=%d> grid=%lld block=%d lds=%zu tile_frames=%d remap=%d",
             type_name<T>(), type_name<A>(), C, P, U, NT, DV, ntiles, WG, lds, TF, xcd_remap);
    return MAVG_OK;
  }
  WideParams p{};
  p.in = sg.in;
  p.out = sg.out;
  p.hist = sg.hist;
  p.nframes = nframes;
  p.ntiles = ntiles;
  p.k = k;
  p.halo_g = (int)Hg;
  p.xk_off = (int)((EPG - ((long long)k * C) % EPG) % EPG);
  p.xcd_remap = xcd_remap;
  p.pre = sg.pre;
  p.o = make_out_params(k);
  if (lds > 64 * 1024) {
    const int s = raise_dyn_lds_limit<&wide_tile_kernel<T, A, C, P, U, WG, NT, DV>>(80 * 1024);
    if (s != MAVG_OK) return s;
  }
  hipLaunchKernelGGL((wide_tile_kernel<T, A, C, P, U, WG, NT, DV>), dim3((unsigned)ntiles), dim3(WG), lds, st, p);
  return hipGetLastError() == hipSuccess ? MAVG_OK : MAVG_ERR_HIP;
}

// the channel-per-lane tile (mavg_wide.hpp chan_tile_kernel): lanes own one
// channel of Q frames; same stage, halo and workspace-free launch as the wide tile
// IPOK: with XG and a staged halo of exactly k frames (k C elements fill whole 256-B rows), the
// in-place output form (chan_tile_kernel IP).  In-process (profiles/r05_tuning/wide/ip_*): fp32
// C = 4 k=2048 0.737 -> 0.756; fp32 C = 8 k=1024 0.750 -> 0.746 and int16 C = 8 k=2048 0.649 ->
// 0.485 (170 VGPRs, 2 workgroups per CU), so only fp32 C = 4 asks for it
// XL: x as 16-B frame-piece loads plus quad transposes (mavg_wide.hpp xl_load; XG only)
template <typename T, typename A, int C, int Q, int WG, int NT, int DV = 0, bool XG = false, bool IPOK = false,
          int XL = 0>
int launch_chan_tile(const Sig& sg, int k, hipStream_t st, int xcd_remap = kRemapGroup) {
  constexpr int EPG = 16 / (int)sizeof(T);
  constexpr int NW = WG / 64;
  constexpr int CL = C * (int)sizeof(T) / 4;  // dword columns per frame (a lane's)
  constexpr int TF = NW * (64 / CL) * Q;      // waves x frame blocks x frames per block
  constexpr int TG = TF * C / EPG;
  const long long nframes = sg.nframes;
  const long long hg = ((long long)k * C + EPG - 1) / EPG;  // granules covering the k-frame halo
  const long long Hg = (hg + 15) / 16 * 16;                // whole 256-B LDS rows
  if (XG && (long long)k < TF) return MAVG_ERR_UNSUPPORTED;  // x[n-k] must lie in the halo
  const size_t lds = (size_t)(Hg + (XG ? 0 : TG)) * 16 + (size_t)2 * NW * C * sizeof(A);
  if (lds > 80 * 1024) return MAVG_ERR_UNSUPPORTED;
  const long long ntiles = (nframes + TF - 1) / TF;
  if (ntiles > 0x7fffffffLL) return MAVG_ERR_UNSUPPORTED;
  const bool ip = XG && IPOK && Hg * EPG == (long long)k * C;  // staged halo frames Hg EPG / C == k
  if (g_plan) {
    snprintf(g_plan->text, sizeof(g_plan->text),
             "chan_tile<%s,acc=%s,C=%d,Q=%d,nt=%d,dv=%d%s%s%s> grid=%lld block=%d lds=%zu tile_frames=%d remap=%d",
             type_name<T>(), type_name<A>(), C, Q, NT, DV, XG ? ",xg=1" : "", ip ? ",ip=1" : "", XL ? ",xl=1" : "",
             ntiles, WG, lds, TF,
             xcd_remap);
    return MAVG_OK;
  }
  WideParams p{};
  p.in = sg.in;
  p.out = sg.out;
  p.hist = sg.hist;
  p.nframes = nframes;
  p.ntiles = ntiles;
  p.k = k;
  p.halo_g = (int)Hg;
  p.xk_off = 0;
  p.xcd_remap = xcd_remap;
  p.pre = sg.pre;
  p.o = make_out_params(k);
  auto launch = [&](auto ipc) -> int {
    constexpr bool IP = decltype(ipc)::value;
    if (lds > 64 * 1024) {
      const int s = raise_dyn_lds_limit<&chan_tile_kernel<T, A, C, Q, WG, NT, DV, XG, IP, XL>>(80 * 1024);
      if (s != MAVG_OK) return s;
    }
    hipLaunchKernelGGL((chan_tile_kernel<T, A, C, Q, WG, NT, DV, XG, IP, XL>), dim3((unsigned)ntiles), dim3(WG), lds, st, p);
    return hipGetLastError() == hipSuccess ? MAVG_OK : MAVG_ERR_HIP;
  };
  if constexpr (XG && IPOK) {
    if (ip) return launch(std::true_type{});
  }
  return launch(std::false_type{});
}

// look-ahead scan (one pass over HBM): zero the record granules, then one
// launch whose tile t publishes the records of tile t + ahead and scans
// tile t with its carry from earlier records (mavg_lookback.hpp).
// Workspace: the granule block, at the start of the workspace, padded to
// 16 bytes (the memset's fast form, cdna_hip_programming.md Guideline 16).
constexpr int kAheadSpin = 256;   // polls of an untagged granule before recomputing it
// Test hook (mavg_test_ahead_schedule, include/mavg_debug.h; compiled into
// the debug build only, MAVG_TEST_HOOKS): the parity tests force the
// recompute path with spin 0 and short or absent look-ahead; results are
// bitwise the same for every setting.  -1 = the tuned defaults.  Relaxed
// atomics: no environment reads on the launch path.  The release library has
// no process-wide mutable state.
#ifdef MAVG_TEST_HOOKS
extern std::atomic<int> g_test_ahead_slots;
extern std::atomic<int> g_test_ahead_spin;
#endif
template <typename T, typename A, int C, int F, int U>
constexpr size_t ahead_granule_bytes(long long nrec) {
  using SA = typename ScanAcc<T, A>::type;
  // + 16 bytes of launch statistics (MAVG_AHEAD_STATS builds only)
  return (((size_t)(nrec > 0 ? nrec : 1) * C * GranCount<SA>::n * 8) + 15) / 16 * 16 + 16;
}
// Windows past an XCD's L2 reach (ahead_scan_kernel): window-matched runs,
// remap mode G.  The window is m = k/T tiles; with runs of G tiles a period
// is 8G, and x[n-k]'s tile lies J periods back on the tile's own XCD when
// 8JG ~ m, off by d = |m - 8JG| tiles: a fraction ~d/G of the tiles reads it
// from another XCD.  G <= min(48, D/20) keeps each record's producer (D/8
// slots ahead of its tile) and each run total's (D/8 - 2G) ahead of their
// consumers; among the J that allow it (up to 8 more than the smallest) the
// one with the smallest d/G wins.
constexpr int kAheadRunMax = 48;
inline int ahead_run_length(long long k, int TF, int ahead) {
  const int gmax = std::max(2, std::min(kAheadRunMax, ahead / 20));
  const double m = (double)k / TF;
  int J = 1;
  while (m / (8.0 * J) > gmax + 0.5) ++J;
  int best = 0;
  double best_miss = 2.0;
  for (int j = J; j < J + 8; ++j) {
    const int G = std::max(2, (int)std::lround(m / (8.0 * j)));
    const double miss = std::fabs(m - 8.0 * j * G) / G;
    if (G <= gmax && miss < best_miss - 1e-9) best_miss = miss, best = G;
  }
  return best > 0 ? best : gmax;
}

// ahead: D, the dispatch slots between a record's producer and its tile (a
// multiple of 8; the test hook overrides it)
// Windows past an XCD's L2 reach run in window-matched runs (remap mode G)
// fp32 mono 8192-frame look-ahead tiles up to this many tiles per window
// (beyond: the 4096-frame run-total kernel)
constexpr long long kAheadU8MaxTiles = 1024;
inline bool ahead_past_l2(long long k, int C, int elem, int TF) {
  return k * C * elem > (1LL << 21) && k >= 8LL * TF;
}
// The windows that take the aggregate-first look-ahead (dispatch_ahead; 16-B units, 32-KiB
// tiles of U = 8 x 256 threads): int16 mono / stereo past a 16-KiB halo, int16 4 channels past
// 64 KiB, fp32 stereo past 32 KiB (the wide tile's), each short of the L2 reach (window-matched
// runs take over there) and int16 mono up to k = 131072 (5e5 measured 0.641 -> 0.624).
template <typename T, int C>
inline bool agg_first_range(long long k) {
  constexpr int F = 16 / (C * (int)sizeof(T));
  constexpr int TF8 = kWG * F * 8;
  const long long halo = k * C * (long long)sizeof(T);
  if (ahead_past_l2(k, C, sizeof(T), TF8)) return false;
  if constexpr (sizeof(T) == 2 && C <= 2) return halo > 16384 && (C == 2 || k <= 131072);
  if constexpr (sizeof(T) == 2 && C == 4) return halo > 65536;
  if constexpr (sizeof(T) == 4 && C == 2) return halo > 32768;
  return false;
}

template <typename T, typename A, int C, int F, int U, int NT, bool RC, bool DMA, bool WREC, int DV = 0, bool HS = false,
          bool RUNS = false, int WG = kWG>
// lds_floor: the LDS the launch allocates at least (fewer workgroups per CU, a footprint cap; 0: none)
int launch_ahead_scan(const Sig& sg, int k, hipStream_t st, Workspace ws, int ahead, bool self = false,
                      size_t lds_floor = 0) {
  constexpr int NW = WG / 64;
  const long long nframes = sg.nframes;
  ahead &= ~7;
  // the tuned D sets the run length G below; the test hook changes only the
  // producer distance, so a forced schedule keeps the plan's tile -> XCD
  // mapping and run-total grouping (the same decomposition, the same bits)
  const int ahead_plan = ahead;
  int spin = kAheadSpin;
#ifdef MAVG_TEST_HOOKS
  {
    const int t = g_test_ahead_slots.load(std::memory_order_relaxed);
    if (t >= 0) ahead = t & ~7;
  }
  {
    const int t = g_test_ahead_spin.load(std::memory_order_relaxed);
    if (t >= 0) spin = t;
  }
#endif
  // one contiguous run per XCD (remap mode 1: x[n-k] is then an L2 hit of the
  // same XCD) while the window's bytes fit comfortably in an XCD's 4 MB L2;
  // past that, 8 separate runs would fetch x[n-k] from the MALL: window-
  // matched runs (ahead_run_length), the chip streaming one front, no head duty.
  // Measured, 2^30 fp32 (profiles/r03_tuning/remap/, period/): one run per
  // XCD -> runs of 64 tiles -> window-matched runs: k=4e6 0.185 -> 0.526;
  // k=1e6 0.524 -> 0.588 -> 0.668; k=6e5 0.594 -> 0.599 -> 0.681
  constexpr int TF = WG * F * U;
  const int xcd_remap = ahead_past_l2(k, C, sizeof(T), TF) ? ahead_run_length(k, TF, ahead_plan) : 1;
  if (RUNS && xcd_remap == 1) return MAVG_ERR_UNSUPPORTED;
  constexpr int VE = F * C;
  constexpr int NSEG = U * NW;
  using SA = typename ScanAcc<T, A>::type;
  constexpr size_t kStageBytes = (((size_t)(U * WG + 1) * VE * sizeof(T)) + 15) & ~(size_t)15;
  const long long ntiles = (nframes + TF - 1) / TF;
  const long long nfull = nframes / TF;
  if (ntiles > 0x7fffffffLL) return MAVG_ERR_UNSUPPORTED;
  // runs with a published total: run r's is published with the record of
  // the last tile of run r + 8, which must be a whole tile of a complete
  // period (remap_tile maps the blocks past those to themselves)
  const long long P = xcd_remap > 1 ? ntiles / (8LL * xcd_remap) : 0;
  const long long pub_periods = P - 1 - (8LL * xcd_remap * P > nfull ? 1 : 0);
  const long long runs_done = RUNS && pub_periods > 0 ? 8 * pub_periods : 0;
  const size_t rec_bytes = ahead_granule_bytes<T, A, C, F, U>(nfull * (WREC ? NW : 1)) - 16;
  const size_t run_bytes = ((size_t)runs_done * C * GranCount<A>::n * 8 + 15) / 16 * 16;
#ifdef MAVG_AHEAD_TRACE
  const size_t trace_bytes = (size_t)ntiles * 64;  // tuning builds: 8 stamps per tile, after the stats
#else
  const size_t trace_bytes = 0;
#endif
  const size_t need = rec_bytes + run_bytes + 16 + trace_bytes;
  size_t lds = kStageBytes + (size_t)NW * C * sizeof(A) + (size_t)(NSEG + 3 * NW) * C * sizeof(SA);
  if (HS) lds = (lds + 15) / 16 * 16 + (size_t)U * WG * VE * sizeof(T);  // + the tile
  if (lds > kLdsBudget) return MAVG_ERR_UNSUPPORTED;
  lds = std::max(lds, lds_floor);
  if (g_plan) {
    snprintf(g_plan->text, sizeof(g_plan->text),
             "ahead_scan<%s,acc=%s,C=%d,F=%d,U=%d,%s,nt=%d,rc=%d,dma=%d,wrec=%d,dv=%d> grid=%lld block=%d lds=%zu "
             "tile_frames=%d ahead=%d remap=%d%s%s ws=%zu",
             type_name<T>(), type_name<A>(), C, F, U, HS ? "hillis" : "blelloch", NT, (int)RC, (int)DMA, (int)WREC, DV,
             ntiles, WG, lds, TF, ahead, xcd_remap, RUNS ? " runs=1" : "", self ? " self=1" : "", need);
    g_plan->ws_bytes = need;
    return MAVG_OK;
  }
  if (ws.ptr == nullptr || ws.bytes < need) return MAVG_ERR_WORKSPACE;
  if ((reinterpret_cast<uintptr_t>(ws.ptr) & 15u) != 0) return MAVG_ERR_MISALIGNED;
  if (hipMemsetAsync(ws.ptr, 0, need, st) != hipSuccess) return MAVG_ERR_HIP;
  AheadParams p{};
  p.in = sg.in;
  p.out = sg.out;
  p.hist = sg.hist;
  p.nframes = nframes;
  p.pre = sg.pre;
  p.eio = sg.eio;
  p.nfull = nfull;
  p.k = k;
  p.o = make_out_params(k);
  p.halo_units = (k + F - 1) / F;
  p.xk_off = (int)((VE - ((long long)k * C) % VE) % VE);
  p.xcd_remap = xcd_remap;
  p.runs_done = runs_done;
  p.ahead = ahead;
  p.head = xcd_remap == 1 ? (int)std::min<long long>((long long)k / TF, nfull) : 0;  // head duty: mode 1 only
  p.spin = spin;
  p.self = self ? 1 : 0;
  p.gran = static_cast<unsigned long long*>(ws.ptr);
  p.runs = reinterpret_cast<unsigned long long*>(static_cast<unsigned char*>(ws.ptr) + rec_bytes);
  p.stats = static_cast<unsigned char*>(ws.ptr) + need - trace_bytes - 16;
#ifdef MAVG_AHEAD_TRACE
  p.trace = reinterpret_cast<unsigned long long*>(static_cast<unsigned char*>(ws.ptr) + need - trace_bytes);
#endif
  hipLaunchKernelGGL((ahead_scan_kernel<T, A, C, F, U, NT, RC, DMA, WREC, DV, HS, RUNS, WG>), dim3((unsigned)ntiles),
                     dim3(WG), lds, st, p);
  return hipGetLastError() == hipSuccess ? MAVG_OK : MAVG_ERR_HIP;
}

// The look-ahead scan's shape for the dtype, channel count and window
// (tools/tune/sweep_long.sh, 2^30 samples, k=44100): 4096-frame
// tiles (U=4 x 16-B units), LDS-DMA stage, non-temporal stage loads and
// output stores (nt=9).
//   mono (fp32, int16): per-wave records published early (WREC) while a
//     window's records fit one round of loads (k/T < 64), D = 512 slots;
//     fp32 keeps the tile in registers across the second barrier (RC, fewer
//     live fp64 accumulators)
//   otherwise: per-tile records, D = 768 (stereo int16) / 1024
template <typename T, typename A, int C, int F, bool HS = false, int U0 = 4>
int dispatch_ahead(const Sig& sg, int k, hipStream_t st, Workspace ws) {
  constexpr int WG = kWG;
  constexpr int U = U0;
  constexpr int TF = WG * F * U;
  constexpr int kNtA = kNtStore | kNtHalo;
  constexpr bool kRC = sizeof(T) == 4 && C == 1 && !HS;
  constexpr int D = C == 2 ? 768 : 1024;
  int s = MAVG_ERR_UNSUPPORTED;
  // self-published records (AheadParams::self) for fp32 mono windows of at most 3 tiles: no phase A,
  // the records of the few tiles a window spans are out by the time the scan is done (A/B,
  // profiles/r03_tuning/self/: k=5000 0.704 -> 0.734, 8192 0.712 -> 0.735, 12288 0.709 -> 0.728;
  // k=20000 0.712 -> 0.692 and int16 stereo / mono past 3 tiles lose: late neighbours' records)
  const bool self = sizeof(T) == 4 && C == 1 && !HS && (long long)k <= 3LL * TF;
  // 8192-frame tiles (U = 8, 32 KiB) with per-tile records: 3 workgroups per
  // CU with twice the bytes each instead of 5-6 with 16 KiB, and a shorter
  // look-ahead in slots (fp32 D = 320, int16 D = 256) for about the same
  // prefetch in bytes.  Kept where bench.py's timing shows the gain
  // (tools/tune/ab_libs.py against -DMAVG_AHEAD_NO_U8, profiles/r04_tuning/u8/):
  //   fp32 mono past the L2 reach (window-matched runs), up to 1024 tiles,
  //     without run totals: k=2e6 0.613 -> 0.650, 4e6 0.589 -> 0.621, 1e6
  //     0.657 -> 0.660; shorter fp32 windows lose (k=44100 0.703 -> 0.684,
  //     20000 0.690 -> 0.674) and keep the 4096-frame per-wave records;
  //   int16 stereo short of the run-total range: k=44100 0.629 -> 0.643,
  //     1e5 0.527 -> 0.572.
  //   int16 mono (16384-frame tiles) lost in the tuner (0.680 -> 0.667).
  // (16-B units only: the frame-unit form of element-aligned views keeps U = 4)
  // Aggregate-first records (round 6): int16 mono / stereo / 4 channels and fp32 stereo take
  // 32-KiB tiles (U = 8 x 256 threads: 16384 / 8192 / 4096 frames) with self-published records --
  // no phase A; each tile publishes its own aggregate as soon as its loads land, and the carry reads
  // the records after its in-tile scan.  With tiles this long a window spans few of them, and the
  // nearest ones are out before the scan is done; with 4096-frame mono tiles the same mode loses
  // (round 3, and again here).  In-process A/B against the library's dispatch, 2^30 samples,
  // fraction of 8 TB/s (tools/tune/wide_ab.hip "self", profiles/r06_tuning/self/):
  //   int16 mono   k=10000 0.711 -> 0.730 (the 1024-thread tile), 12000 0.706 -> 0.733, 20000
  //                0.647 -> 0.673, 44100 0.666 -> 0.698, 1e5 0.638 -> 0.648, 2e5 0.638 -> 0.640
  //                (k <= 131072 here), 5e5 0.641 -> 0.624; the tile keeps k <= 8192 (0.756 vs 0.734)
  //   int16 stereo k=8192 0.657 -> 0.711, 12000 0.614 -> 0.714, 44100 0.640 -> 0.702, 2e5 0.574 ->
  //                0.702; the tile keeps k <= 4096 (0.747 vs 0.716)
  //   int16 C = 4  k=20000 0.607 -> 0.628, 44100 0.597 -> 0.626, 1e5 0.484 -> 0.619 (against the
  //                wide look-ahead, and the 4096-frame look-ahead past int32 sums); k=8192 a tie
  //   fp32 stereo  k=20000 0.661 -> 0.691, 44100 0.651 -> 0.689, 1e5 0.647 -> 0.691 (against the
  //                wide look-ahead)
  // Not taken: fp32 mono (k=20000 0.730 vs 0.696, 44100 0.718 vs 0.688), fp32 / int16 with 4 / 8
  // channels in 1-frame units (0.42 / 0.48 against the channel-per-lane look-ahead's 0.62 / 0.59),
  // the Hillis-Steele flavour (k=44100 0.593 vs 0.574).
  constexpr bool kAgg = !HS && U0 == 4 && F * C * (int)sizeof(T) == 16 &&
                        ((sizeof(T) == 2 && C <= 4) || (sizeof(T) == 4 && C == 2));
  if constexpr (kAgg) {
    if (agg_first_range<T, C>(k))
      return launch_ahead_scan<T, A, C, F, 8, kNtA, false, true, false, 0, false, false, WG>(sg, k, st, ws, 256, true);
  }
  // Past the L2 reach (window-matched runs, remap mode G): fp32 mono and int16 mono / stereo in
  // the same 32-KiB tiles without run totals up to 1024 tiles per window.  Round 6: int16 with
  // self-published records (int16 mono only up to k = 2^21), fp32 mono keeping phase A.  There D
  // only bounds the run length (G <= D/20; the records a carry reads are J periods old): 320,
  // 960 for int16 stereo past 2^21.  The in-process tuner favoured self-publication for fp32 too
  // (k=1e6 0.675 -> 0.713, 4e6 0.645 -> 0.664) but bench.py's own timing did not: the release
  // library against a phase-A build in bench.py's environment (tools/tune/ab_libs.py,
  // tools/gpu/r06_far_ab.sh, profiles/r06_tuning/far/), self-published vs phase A: fp32 mono
  // k=6e5 0.673 vs 0.692, 1e6 0.674 vs 0.684, 2e6 0.662 vs 0.673, 4e6 0.570 vs 0.639; int16 mono
  // 1.5e6 0.634 vs 0.605, stereo 6e5 0.608 vs 0.584, 2e6 0.599 vs 0.577 (outputs bitwise equal).
  constexpr bool kFar = !HS && U0 == 4 && F * C * (int)sizeof(T) == 16 && (C == 1 || (sizeof(T) == 2 && C == 2));
  if constexpr (kFar) {
    constexpr int TF8 = WG * F * 8;
    if (ahead_past_l2(k, C, sizeof(T), TF8) && (long long)k <= kAheadU8MaxTiles * TF8) {
      const bool far_self = sizeof(T) == 2 && !(C == 1 && k > (1 << 21));
      const int far_d = sizeof(T) == 2 && C == 2 && k > (1 << 21) ? 960 : 320;
      return launch_ahead_scan<T, A, C, F, 8, kNtA, kRC, true, false, 0, false, false, WG>(sg, k, st, ws, far_d,
                                                                                        far_self);
    }
  }
  constexpr bool kU8 = !HS && U0 == 4 && F * C * (int)sizeof(T) == 16 && sizeof(T) == 2 && C == 2;
  if constexpr (kU8) {
    // (int16 stereo windows that reach here short of the run-total range: the reference block
    // size's fallbacks; the tuned dispatch takes the tiles or the aggregate-first form)
    const bool u8 = !(ahead_past_l2(k, C, sizeof(T), TF) && (long long)k > 384LL * TF);
    // phase A keeps the default policy: non-temporal phase-A loads (kNtPhaseA) measured +3-4 % in
    // the in-process tuner but -15 to -18 % in bench.py's timing (round 4, profiles/r04_tuning/u8/
    // nta_*, bench_timing_nta_*: k=4e6 0.620 -> 0.510, 2e6 0.652 -> 0.546, 1e6 0.660 -> 0.556)
    constexpr int kNt8 = kNtA;
    if (u8) return launch_ahead_scan<T, A, C, F, 8, kNt8, kRC, true, false, 0, false, false, WG>(sg, k, st, ws, 256);
  }
  // per-wave records: mono only (instantiated for C = 1 alone)
  const bool wrec = C == 1 && (long long)k / TF + 1 <= 64;
  if (wrec) {
    if constexpr (C == 1) s = launch_ahead_scan<T, A, C, F, U, kNtA, kRC, true, true, 0, HS, false, WG>(sg, k, st, ws, 512, self);
  }
  // run totals (O(J + G) carry items instead of k/T) where the windows are
  // long enough to pay for the kernel's extra registers (4 waves per SIMD
  // instead of 5): > 384 tiles (A/B, profiles/r03_tuning/runs/: fp32
  // k=4e6 0.543 -> 0.596, k=2e6 0.623 -> 0.641; k=1e6 0.670 -> 0.642)
  else if (C <= 2 && U0 == 4 && !HS && ahead_past_l2(k, C, sizeof(T), TF) && (long long)k > 384LL * TF)
    s = launch_ahead_scan<T, A, C, F, U, kNtA, kRC, true, false, 0, HS, C <= 2 && U0 == 4 && !HS, WG>(sg, k, st, ws, D);
  else
    s = launch_ahead_scan<T, A, C, F, U, kNtA, kRC, true, false, 0, HS, false, WG>(sg, k, st, ws, D, self);
  // the Hillis-Steele form also stages the tile: wide frames (e.g. 8 fp32
  // channels, 32 B) take half tiles to stay inside the LDS budget
  if constexpr (HS && U0 > 2) {
    if (s == MAVG_ERR_UNSUPPORTED) return dispatch_ahead<T, A, C, F, HS, U0 / 2>(sg, k, st, ws);
  }
  return s;
}

// wide look-ahead scan (mavg_wide.hpp): the look-ahead record carry in its
// unit layout (F frames x U units per lane, per-tile records) with the wide
// in-tile scan (P-frame chunks x UW rows); 16-B-aligned views only.
// self: aggregate-first (self-published) records, the halo-only CH form only (wide_ahead_kernel: every
// producer forms a record in one order, so fp32 records keep their bits too)
template <typename T, typename A, int C, int P, int UW, int WG, int NT, int DV, int F, int U, bool CH = false,
          bool XG = false, int MW = 0, int XL = 0>
int launch_wide_ahead(const Sig& sg, int k, hipStream_t st, Workspace ws, int ahead, bool self = false) {
  // (self + XL: the self-published record would be summed before the quad transposes)
  if (self && !(CH && XG && XL != 1)) return MAVG_ERR_UNSUPPORTED;
  if (XL == 2 && !self) return MAVG_ERR_UNSUPPORTED;  // XL = 2: the columns formed before the self-published record
  constexpr int NW = WG / 64;
  constexpr int EPG = 16 / (int)sizeof(T);
  constexpr int CL = C * (int)sizeof(T) / 4 > 0 ? C * (int)sizeof(T) / 4 : 1;  // CH: dword columns per frame
  constexpr int TF = CH ? NW * (64 / CL) * P : WG * P * UW;  // CH: P frames of one dword column per lane
  constexpr int TG = TF * C / EPG;
  constexpr int NSEG = UW * NW;
  using SA = typename ScanAcc<T, A>::type;
  const long long nframes = sg.nframes;
  ahead &= ~7;
  const int ahead_plan = ahead;
  int spin = kAheadSpin;
#ifdef MAVG_TEST_HOOKS
  {
    const int t = g_test_ahead_slots.load(std::memory_order_relaxed);
    if (t >= 0) ahead = t & ~7;
  }
  {
    const int t = g_test_ahead_spin.load(std::memory_order_relaxed);
    if (t >= 0) spin = t;
  }
#endif
  const int xcd_remap = ahead_past_l2(k, C, sizeof(T), TF) ? ahead_run_length(k, TF, ahead_plan) : 1;
  const long long ntiles = (nframes + TF - 1) / TF;
  const long long nfull = nframes / TF;
  if (ntiles > 0x7fffffffLL) return MAVG_ERR_UNSUPPORTED;
#ifdef MAVG_AHEAD_TRACE
  const size_t trace_bytes = (size_t)ntiles * 64;  // tuning builds: 8 stamps per tile, after the stats
#else
  const size_t trace_bytes = 0;
#endif
  const size_t need = ahead_granule_bytes<T, A, C, F, U>(nfull) + trace_bytes;  // per-tile records + 16
  // the shifted tile (+ one granule for an x[n-k] extraction) and, unless XG, the tile
  const size_t lds = (size_t)((XG ? 1 : 2) * TG + 1) * 16 + (size_t)NW * C * sizeof(A) +
                     (size_t)(NSEG + 3 * NW) * C * sizeof(SA);
  if (lds > 80 * 1024) return MAVG_ERR_UNSUPPORTED;
  if (g_plan) {
    snprintf(g_plan->text, sizeof(g_plan->text),
             "wide_ahead<%s,acc=%s,C=%d,P=%d,U=%d,nt=%d,dv=%d,F=%d,FU=%d%s%s,mw=%d,xl=%d> grid=%lld block=%d lds=%zu "
             "tile_frames=%d ahead=%d remap=%d%s ws=%zu",
             type_name<T>(), type_name<A>(), C, P, UW, NT, DV, F, U, CH ? ",ch=1" : "", XG ? ",xg=1" : "", MW, XL, ntiles,
             WG, lds, TF, ahead, xcd_remap, self ? " self=1" : "", need);
    g_plan->ws_bytes = need;
    return MAVG_OK;
  }
  if (ws.ptr == nullptr || ws.bytes < need) return MAVG_ERR_WORKSPACE;
  if ((reinterpret_cast<uintptr_t>(ws.ptr) & 15u) != 0) return MAVG_ERR_MISALIGNED;
  if (hipMemsetAsync(ws.ptr, 0, need, st) != hipSuccess) return MAVG_ERR_HIP;
  AheadParams p{};
  p.in = sg.in;
  p.out = sg.out;
  p.hist = sg.hist;
  p.nframes = nframes;
  p.pre = sg.pre;
  p.eio = 0;
  p.nfull = nfull;
  p.k = k;
  p.o = make_out_params(k);
  p.halo_units = (k + F - 1) / F;
  p.xk_off = (((F - k % F) % F) * C) % EPG;
  p.xcd_remap = xcd_remap;
  p.runs_done = 0;
  p.ahead = ahead;
  p.head = xcd_remap == 1 ? (int)std::min<long long>((long long)k / TF, nfull) : 0;
  p.spin = spin;
  p.self = self ? 1 : 0;
  p.gran = static_cast<unsigned long long*>(ws.ptr);
  p.runs = nullptr;
  p.stats = static_cast<unsigned char*>(ws.ptr) + need - trace_bytes - 16;
#ifdef MAVG_AHEAD_TRACE
  p.trace = reinterpret_cast<unsigned long long*>(static_cast<unsigned char*>(ws.ptr) + need - trace_bytes);
#endif
  if (lds > 64 * 1024) {
    const int s = raise_dyn_lds_limit<&wide_ahead_kernel<T, A, C, P, UW, WG, NT, DV, F, U, CH, XG, MW, XL>>(80 * 1024);
    if (s != MAVG_OK) return s;
  }
  hipLaunchKernelGGL((wide_ahead_kernel<T, A, C, P, UW, WG, NT, DV, F, U, CH, XG, MW, XL>), dim3((unsigned)ntiles), dim3(WG), lds,
                     st, p);
  return hipGetLastError() == hipSuccess ? MAVG_OK : MAVG_ERR_HIP;
}

// Algorithm selection for the scan family (measured on MI355X with
// tools/tune/tune_scan.hip + tools/tune/sweep_*.sh, 2^30 samples, back-to-back
// launches; DESIGN.md "Tuning").  Tiles are 4 KiB of samples per U.
//   Blelloch flavour, by halo bytes H = k*C*elem (nt: every load and store
//   non-temporal; ntS: the split policy kNtS below):
//     int16  H <= 256: U2 nt | H <= 4 KiB: U4 nt | H <= 8 KiB: U4 ntS |
//            H <= 16 KiB: U4 x 512 threads ntS | H <= ~47 KiB: U2 x 1024 (80 KiB LDS) ntS
//     fp32   mono H <= 512: U2 nt rc | H <= 4 KiB: U2 ntS rc | H <= 8 KiB: U2 x 512 ntS rc |
//            H <= 16 KiB: U4 x 512 ntS rc
//     longer windows (fp32 H > 16 KiB, int16 past the 1024-thread tile): the
//     look-ahead scan (dispatch_ahead; needs the workspace)
//   Hillis-Steele flavour: the halo-staged tile while it fits LDS (fp32: U4 nt
//   for H <= 512 B, else U8 ntS; int16: U4 x 512 threads ntS), then the
//   look-ahead scan with the Hillis-Steele in-tile scan (needs the workspace).
template <typename T, typename A, int C, int F, bool HS>
int dispatch_scan_f(const Sig& sg, int k, int block, hipStream_t st, Workspace ws) {
  constexpr int VE = F * C;
  constexpr int kUnitBytes = VE * (int)sizeof(T);
  const long long halo_bytes = (long long)k * C * (long long)sizeof(T);
  auto tile_lds = [&](int U, int WG = kWG) -> long long {
    const long long hu = (k + F - 1) / F;
    return (hu + (long long)U * WG + 1) * kUnitBytes + (U * (WG / 64) + WG / 64) * C * (long long)sizeof(A);
  };
  auto fits = [&](int U, int WG) { return tile_lds(U, WG) <= (long long)lds_budget(WG); };
  constexpr long long kB = (long long)kLdsBudget;
  constexpr int kNt = kNtLoad | kNtStore;
  // split policy: nt tile loads except the tail the next tile's halo re-reads,
  // nt halo loads (their last use), nt stores (tools/tune/sweep_nt.sh: +1-4 %
  // over default-policy loads wherever the halo is re-read from L2)
  constexpr int kNtS = kNtSplit | kNtHalo | kNtStore;
  if (block != 0) {
    // the reference's block size: a U=2 tile of block_wg(block) threads while
    // its halo fits that workgroup's LDS, else the tuned dispatch below (the
    // plan string shows the workgroup that runs)
    const int wg = block_wg(block);
    constexpr bool kR = sizeof(T) == 4;  // RC as in the tuned rules (fp32 on, int16 off)
    if (wg == 64 && fits(2, 64)) return launch_tile_scan<T, A, C, F, 2, HS, kNtS, 64, kR>(sg, k, st);
    if (wg == 128 && fits(2, 128)) return launch_tile_scan<T, A, C, F, 2, HS, kNtS, 128, kR>(sg, k, st);
    if (wg == 256 && fits(2, 256)) return launch_tile_scan<T, A, C, F, 2, HS, kNtS, 256, kR>(sg, k, st);
    if (wg == 512 && fits(2, 512)) return launch_tile_scan<T, A, C, F, 2, HS, kNtS, 512, kR>(sg, k, st);
    if (wg == 1024 && fits(2, 1024)) return launch_tile_scan<T, A, C, F, 2, HS, kNtS, 1024, kR>(sg, k, st);
  }
  if constexpr (!HS && sizeof(T) == 4 && C == 4 && F == 2) {
    // fp32 4 channels in 32-B units (dispatch_scan_c): 1024-frame tiles up to
    // 4 KiB of halo, then the look-ahead scan in 1024-frame tiles (in-process
    // A/B against 1-frame units, profiles/r03_tuning/c4/: k=7 0.46 -> 0.64,
    // k=200 0.45 -> 0.65, k=2000 0.41 -> 0.50, k=44100 0.40 -> 0.48)
    if (halo_bytes <= 4096 && fits(2, kWG)) return launch_tile_scan<T, A, C, F, 2, false, kNtS, kWG, true>(sg, k, st);
    return dispatch_ahead<T, A, C, F, false, 2>(sg, k, st, ws);
  }
  if constexpr (!HS && sizeof(T) == 4 && C == 8 && F == 2) {
    // fp32 8 channels in 64-B units (2 frames per lane, 4 x 16-B accesses), past
    // the LDS-staged halo only (dispatch_scan_c): the look-ahead scan in 512-frame
    // tiles (profiles/r03_tuning/c8/: k=300 0.208 -> 0.267, k=1024 0.198 -> 0.238, k=44100 0.180 -> 0.208)
    return dispatch_ahead<T, A, C, F, false, 1>(sg, k, st, ws);
  }
  if constexpr (!HS) {
    // RC (in-lane prefix rebuilt after the barrier): on for fp32, off for
    // int16 (measured both ways, tools/tune/ab_rc.sh, sweep_lookback2.sh).
    // Longer halos take bigger workgroups: the LDS stage per workgroup then
    // carries more waves (tools/tune/sweep_wg.sh, sweep_wg2.sh).
    if constexpr (sizeof(T) == 2) {
      // past a 16-KiB halo int16 mono / stereo take the aggregate-first look-ahead
      // (dispatch_ahead, round 6) instead of the 1024-thread tile
      if constexpr (kUnitBytes == 16 && C <= 2) {
        if (block == 0 && agg_first_range<T, C>(k)) return dispatch_ahead<T, A, C, F>(sg, k, st, ws);
      }
      // int16 keeps register staging: LDS-DMA tiles won the in-process tuner's
      // A/B (mono U2 x 512 0.811-0.820 vs 0.800-0.803) but lost 2-3.5 % in
      // bench.py's own timing, one HIP-event pair per back-to-back launch
      // (tools/tune/ab_libs.py, profiles/r02_tuning/r02_ablibs*); stereo tied
      if (halo_bytes <= 256 && fits(2, kWG))
        return launch_tile_scan<T, A, C, F, 2, false, kNt, kWG, false>(sg, k, st);
      if (halo_bytes <= 4096 && fits(4, kWG))
        return launch_tile_scan<T, A, C, F, 4, false, kNt, kWG, false>(sg, k, st);
      if (halo_bytes <= 8192 && fits(4, kWG))
        return launch_tile_scan<T, A, C, F, 4, false, kNtS, kWG, false>(sg, k, st);
      if (halo_bytes <= 16384 && fits(4, 512))
        return launch_tile_scan<T, A, C, F, 4, false, kNtS, 512, false>(sg, k, st);
      if (fits(2, 1024))
        return launch_tile_scan<T, A, C, F, 2, false, kNtS, 1024, false>(sg, k, st);
    } else {
      // fp32 mono (round 2): the halo and the tile staged by LDS-DMA, 512-thread
      // workgroups (2^30 samples, fraction of peak, in-process A/B against the
      // round-1 rules: k=64 0.825 vs 0.802, k=256 0.819 vs 0.795, k=1024 0.810
      // vs 0.801, k=2048 0.801 vs 0.794, k=4096 0.788 vs 0.778;
      // profiles/r02_tuning/r02_tdma*); confirmed in bench.py's timing
      // (tools/tune/ab_libs.py, r02_ablibs2): k=64 0.814 vs 0.780, k=1024 0.802
      // vs 0.797, k=4096 0.781 vs 0.773 against the same tiles register-staged
      constexpr bool kD = true;
      constexpr int kDV = 0;
      if (C == 1 && halo_bytes <= 8192 && fits(2, 512))
        return launch_tile_scan<T, A, C, F, 2, false, kNtS, 512, true, kDV, kD>(sg, k, st);
      if (C == 1 && halo_bytes <= 16384 && fits(4, 512))
        return launch_tile_scan<T, A, C, F, 4, false, kNtS, 512, true, kDV, kD>(sg, k, st);
      if (C == 1 && halo_bytes <= 512 && fits(2, kWG))
        return launch_tile_scan<T, A, C, F, 2, false, kNt, kWG, true>(sg, k, st);
      if (halo_bytes <= 4096 && fits(2, kWG))
        return launch_tile_scan<T, A, C, F, 2, false, kNtS, kWG, true>(sg, k, st);
      if (halo_bytes <= 8192 && fits(2, 512))
        return launch_tile_scan<T, A, C, F, 2, false, kNtS, 512, true>(sg, k, st);
      if (halo_bytes <= 16384 && fits(4, 512))
        return launch_tile_scan<T, A, C, F, 4, false, kNtS, 512, true>(sg, k, st);
      // fp32 halos past 16 KiB: the look-ahead scan beats the 1024-thread
      // tile (k=8192: 0.73 vs 0.69; k=12000: 0.71 vs 0.64, sweep_ahead.sh)
    }
    return dispatch_ahead<T, A, C, F>(sg, k, st, ws);
  } else {
    // Hillis-Steele: the element-wise log-step scans make a tile's compute
    // long, so bigger tiles (fewer halos and barriers per byte) and the split
    // cache policy win (tools/tune/sweep_hillis.sh: fp32 k=1024 0.66 -> 0.78)
    if constexpr (sizeof(T) == 2) {
      if (fits(4, 512))
        return launch_tile_scan<T, A, C, F, 4, HS, kNtS, 512>(sg, k, st, kRemapGroup);
    } else {
      if (C == 1 && halo_bytes <= 512 && fits(4, kWG))
        return launch_tile_scan<T, A, C, F, 4, HS, kNt>(sg, k, st, kRemapGroup);
      if (fits(8, kWG))
        return launch_tile_scan<T, A, C, F, 8, HS, kNtS>(sg, k, st, kRemapGroup);
    }
    (void)kB;
    // past the LDS-staged halo: the look-ahead scan's record carry with the
    // Hillis-Steele in-tile scan (the segment kernel re-read x[n-k] from
    // global memory beyond its LDS ring: 0.25-0.40 of peak)
    return dispatch_ahead<T, A, C, F, true>(sg, k, st, ws);
  }
}

// The wide-frame kernels (mavg_wide.hpp) for multi-channel frames: the wide
// tile while its halo fits the LDS stage, then the wide look-ahead scan;
// MAVG_ERR_UNSUPPORTED where the unit kernels stay (the caller falls back).
// Shapes from in-process A/Bs against the round-3 unit kernels
// (tools/tune/wide_ab.hip, 2^30 samples, fraction of 8 TB/s, mean of
// per-launch events; profiles/r04_tuning/wide/):
//   fp32 C=2  k=7 0.693 -> 0.790 (P8 U1), k=1024 0.645 -> 0.784, k=2048 0.649
//             -> 0.781, k=4096 0.662 -> 0.700 (P16 U1: 4096-frame tiles);
//             look-ahead k=8192 0.646 -> 0.658, k=44100 0.636 -> 0.642 (D=512)
//   fp32 C=4  k=7 0.651 -> 0.776, k=256 0.650 -> 0.794 (P8 U2), k=1024 0.506
//             -> 0.774, k=2048 0.509 -> 0.665 (P8 U1); look-ahead k=4096
//             0.515 -> 0.553, k=44100 ~0.48 -> 0.527 (P4, D=512)
//   fp32 C=8  k=7 0.416 -> 0.794 (P4 x 128 threads), k=256 0.259 -> 0.700,
//             k=512 0.237 -> 0.671, k=1024 0.234 -> 0.537 (P4 U1); look-ahead
//             k=2048 0.236 -> 0.442 (128 threads, D=512), k=44100 0.180 ->
//             0.378 (256 threads, D=1024)
//   int16 C=4 k=7 0.689 -> 0.810 (P8 U1), k=1024 0.711 -> 0.770, k=2048 0.618
//             -> 0.743 (P16 U1); int16 C=8 k=7 0.552 -> 0.798 (P8 x 128
//             threads), k=1024 0.457 -> 0.722, k=2048 0.169 -> 0.591 (P8 U1),
//             look-ahead k=44100 0.400 -> 0.476 (P4)
//   The output division of the int16 wide kernels is the fp64 product (dv=0:
//   int16 C=8 k=1024 P4 0.560 -> 0.602 against the magic multiply).
//   Kept on the unit kernels: fp32 mono and int16 mono/stereo (a tie or a
//   loss: int16 stereo k=1024 0.786 vs 0.788, k=44100 0.631 vs 0.587; fp32
//   mono k=44100 0.677 vs 0.663).
// The 2048-frame halo-only channel-per-lane look-ahead with 16-B frames (fp32 4 channels, int16 8
// channels): self-published records, except fp32 at windows of whole tiles (k mod 2048 = 0), where
// in bench.py's environment phase A measured ahead (k = 8192 0.666-0.670 vs 0.656-0.657, 16384
// 0.670 vs 0.647, 32768 0.666 vs 0.637, 4096 a tie; elsewhere self-published wins by 4-6 %).  int16
// 8 channels: self-published at every window (k = 4096 0.660 vs 0.631, 8192 0.651 vs 0.632,
// 16384 / 32768 ties).  profiles/r06_tuning/xl/ab_f32c4_*, ab_i16c8_*, ab_selfall_*.
template <typename T>
inline bool self_pays(int k) {
  return sizeof(T) == 2 || k % 2048 != 0;  // (int16 8 channels: always)
}

template <typename T, typename A, int C>
int dispatch_wide(const Sig& sg, int k, hipStream_t st, Workspace ws) {
  constexpr int kNtS = kNtSplit | kNtHalo | kNtStore;
  constexpr int kNtA = kNtStore | kNtHalo;
  const long long halo_bytes = (long long)k * C * (long long)sizeof(T);
  if constexpr (sizeof(T) == 4 && C == 2) {
    if (halo_bytes <= 2048) return launch_wide_tile<T, A, C, 8, 1, kWG, kNtS>(sg, k, st);
    if (halo_bytes <= 32768) return launch_wide_tile<T, A, C, 16, 1, kWG, kNtS>(sg, k, st);
    // the unit kernels' aggregate-first look-ahead (dispatch_ahead, round 6) short of the L2 reach
    if (agg_first_range<T, C>(k)) return MAVG_ERR_UNSUPPORTED;
    return launch_wide_ahead<T, A, C, 8, 1, kWG, kNtA, 0, 2, 4>(sg, k, st, ws, 512);
  } else if constexpr (sizeof(T) == 4 && C == 4) {
    // 2048 <= k <= 3584: the halo-only channel-per-lane tile (2048-frame tiles; in-process,
    // profiles/r04_tuning/chan/xg_c4_*, xgr_*: k=2048 0.660 -> 0.712 against the wide tile, 3000
    // 0.541 -> 0.675 against the wide look-ahead; k=4096 ties it, 0.559 vs 0.556)
    // round 6: x of the halo-only forms as 16-B frame loads plus quad transposes (XL, mavg_wide.hpp
    // xl_load) -- a quarter of the vector-memory transactions of the 4-B column loads.  In-process
    // (tools/tune/wide_ab.hip "xl", profiles/r06_tuning/xl/): the look-ahead in 2048-frame tiles
    // (141 VGPRs, D = 384) 0.630-0.639 -> 0.683 at k = 44100, 0.658 -> 0.696 at 20000, 0.6975
    // against the chan tile's 0.683-0.695 at k = 3000 (no in-place form there).  The in-place chan
    // tile (k mod 16 = 0) wins up to k = 3072 (2560: 0.716 vs 0.697, 3072: 0.691 vs 0.686), with XL
    // while four workgroups per CU fit its LDS (k = 2048: 0.728 -> 0.751; k = 2560, three per CU:
    // 0.716 -> 0.704).  1024-frame look-ahead tiles with XL: 0.636-0.671.
    const bool ip = k % 16 == 0;  // the staged halo is exactly k frames (chan tile IP)
    if (k >= 2048 && k <= 3072 && ip) {
      if (halo_bytes <= 40704) return launch_chan_tile<T, A, C, 32, kWG, kNtS, 0, true, true, 1>(sg, k, st);
      // (three workgroups per CU: still ahead of the self-published look-ahead in bench.py's
      // environment, k = 2560 0.718 vs 0.705, 2816 0.709 vs 0.700, 3072 a tie; ab_chan3_*)
      return launch_chan_tile<T, A, C, 32, kWG, kNtS, 0, true, true>(sg, k, st);
    }
    if (halo_bytes <= 4096) return launch_wide_tile<T, A, C, 8, 2, kWG, kNtS>(sg, k, st);
    if (halo_bytes <= 32768) return launch_wide_tile<T, A, C, 8, 1, kWG, kNtS>(sg, k, st);
    // past the chan tile: the halo-only channel-per-lane look-ahead (round 5, in-process,
    // profiles/r05_tuning/wide/pa0_c4_k44100.log: k=44100 0.540 -> 0.593 against the chunk
    // look-ahead), with XL in 2048-frame tiles (above)
    if (self_pays<T>(k)) return launch_wide_ahead<T, A, C, 32, 1, kWG, kNtA, 0, 1, 8, true, true, 0, 2>(sg, k, st, ws, 384, true);
    return launch_wide_ahead<T, A, C, 32, 1, kWG, kNtA, 0, 1, 8, true, true, 0, 1>(sg, k, st, ws, 384);
  } else if constexpr (sizeof(T) == 4 && C == 8) {
    // one channel per lane (chan_tile_kernel, 32 frames each): one scan per
    // tile row for all 8 channels instead of 8 per chunk (in-process A/B,
    // profiles/r04_tuning/chan/: k=1024 0.543 -> 0.566, 512 0.683 -> 0.688,
    // 256 0.705 -> 0.723, 7 0.744 -> 0.778 with 128 threads); past its halo the
    // same in-tile scan in the look-ahead carry (CH): k=2048 0.464 -> 0.488,
    // 4096 0.462 -> 0.487 (128 threads), 44100 0.390 -> 0.433 (256, D = 512)
    if (halo_bytes <= 256) return launch_chan_tile<T, A, C, 32, 128, kNtS>(sg, k, st);
    // windows of at least a tile: stage the halo only, x straight from global memory (XG: half
    // the LDS, twice the workgroups per CU; bench timing, profiles/r04_tuning/chan/bench_timing_xg_*:
    // k=1024 0.562 -> 0.737 (1024-frame tiles, bit-identical), 768 0.583 -> 0.647, 512 0.671 ->
    // 0.739 (512-frame tiles); in-process xg_*: 0.563 -> 0.748, 0.582 -> 0.682, 0.675 -> 0.751)
    // up to 64 KiB of halo (k <= 2048), where the wide look-ahead took over (in-process,
    // profiles/r04_tuning/chan/xgr_*: k=1536 0.478 -> 0.656, 2048 0.482 -> 0.548)
    if (halo_bytes <= 49152 && k >= 1024) return launch_chan_tile<T, A, C, 32, kWG, kNtS, 0, true>(sg, k, st);
    if (halo_bytes <= 32768 && k >= 512) return launch_chan_tile<T, A, C, 32, 128, kNtS, 0, true>(sg, k, st);
    if (halo_bytes <= 32768) return launch_chan_tile<T, A, C, 32, kWG, kNtS>(sg, k, st);
    // past it: the halo-only look-ahead (XG: x straight from global memory, only the shifted tile in
    // LDS, 33 KiB instead of 65 KiB; round 5, in-process, profiles/r05_tuning/wide/pa0_c8_*: k=44100
    // 0.429 -> 0.589 (D = 384), k=2048 0.534 (the halo-only tile) -> 0.616).  256 threads at every
    // such window: with the per-channel totals by butterflies the 128-thread form (512-frame tiles,
    // once +0.5-1 % at k = 1536..4096) ties or loses (in-process, profiles/r05_tuning/wide/
    // after_butterfly/: k=2048 0.672 vs 0.670 on one box, pass12_*: 0.700 vs 0.604 on another)
    return launch_wide_ahead<T, A, C, 32, 1, kWG, kNtA, 0, 1, 4, true, true>(sg, k, st, ws, 384);
  } else if constexpr (sizeof(T) == 2 && C == 4) {
    if constexpr (sizeof(A) == 4) {
      if (halo_bytes <= 8192) return launch_wide_tile<T, A, C, 8, 1, kWG, kNtS>(sg, k, st);
      if (halo_bytes <= 32768) return launch_wide_tile<T, A, C, 16, 1, kWG, kNtS>(sg, k, st);
      // past 64 KiB the unit kernels' aggregate-first look-ahead (dispatch_ahead, round 6)
      if (agg_first_range<T, C>(k)) return MAVG_ERR_UNSUPPORTED;
      // past it the wide look-ahead (64-B chunks, D = 512) instead of the 16-B unit look-ahead
      // (in-process A/B, profiles/r04_tuning/wide/wide_i16_c4_*: k=44100 0.579 -> 0.598, 20000
      // 0.590 -> 0.602; bench timing, bit-exact, profiles/r04_tuning/wide/bench_timing_i16_c4_*:
      // k=44100 0.575 -> 0.586, 60000 0.582 -> 0.591, 20000 0.587 -> 0.590)
      return launch_wide_ahead<T, A, C, 8, 1, kWG, kNtA, 0, 2, 4>(sg, k, st, ws, 512);
    }
  } else if constexpr (sizeof(T) == 2 && C == 8) {
    if constexpr (sizeof(A) == 4) {
      if (halo_bytes <= 256) return launch_wide_tile<T, A, C, 8, 1, 128, kNtS>(sg, k, st);
      if (halo_bytes < 32768) return launch_wide_tile<T, A, C, 8, 1, kWG, kNtS>(sg, k, st);
    }
    // a window of at least the tile (k >= 2048): the halo-only channel-per-lane look-ahead, a dword
    // column (two channels) per lane (int32 sums: k <= 65535), x as 16-B frame pieces (XL) and
    // self-published records (aggregate-first).  In bench.py's environment against the round-5
    // shapes (the halo-only chan tile to k = 3072, then phase A with XL; tools/tune/ab_libs.py,
    // profiles/r06_tuning/xl/ab_i16c8_*, ab_nochan_*, outputs bitwise equal): k = 44100 0.594 ->
    // 0.625, 20000 0.611 -> 0.644, 10000 0.614 -> 0.656, 3072 0.598 -> 0.652, 2560 0.617 -> 0.657,
    // 2048 0.652 -> 0.672 (so int16 no longer takes the chan tile).  (In-process: self-published
    // without XL lost, 0.574 vs 0.596 at k = 44100.)
    if constexpr (sizeof(A) == 4)
      return launch_wide_ahead<T, A, C, 32, 1, kWG, kNtA, 0, 1, 8, true, true, 0, 2>(sg, k, st, ws, 384, true);
    return launch_wide_ahead<T, A, C, 4, 1, kWG, kNtA, 0, 1, 4>(sg, k, st, ws, 1024);
  }
  (void)halo_bytes;
  (void)ws;
  return MAVG_ERR_UNSUPPORTED;
}

template <typename T, typename A, int C>
int dispatch_scan_c(bool vec, bool hs, const Sig& sg, int k, int block, hipStream_t st, Workspace ws) {
  constexpr int VF = (C * (int)sizeof(T) <= 16 && 16 % (C * (int)sizeof(T)) == 0) ? 16 / (C * (int)sizeof(T)) : 0;
  if constexpr ((sizeof(T) == 4 && (C == 2 || C == 4 || C == 8)) || (sizeof(T) == 2 && (C == 4 || C == 8))) {
    if (vec && !hs && !sg.eio && block == 0) {
      const int s = dispatch_wide<T, A, C>(sg, k, st, ws);
      if (s != MAVG_ERR_UNSUPPORTED) return s;
    }
  }
  // fp32 with 8 channels (32-B frames, no vector form): past the 1-frame
  // tiles' LDS-staged halo (8 KiB, k > 256) the look-ahead scan takes 2 frames
  // per lane as well; below it the 1-frame tiles stay (the 64-B-unit tile
  // spills: k=7 0.416 -> 0.383)
  if constexpr (sizeof(T) == 4 && C == 8) {
    if (vec && !hs && !sg.eio && block == 0 && (long long)k * C * (long long)sizeof(T) > 8192)
      return dispatch_scan_f<T, A, C, 2, false>(sg, k, block, st, ws);
  }
  if constexpr (VF > 0) {
    if (vec) {
      // fp32 with 4 channels: a frame is one 16-B unit, so every unit costs 4
      // fp64 wave scans; the Blelloch flavour takes 2 frames (32 B) per lane
      if constexpr (sizeof(T) == 4 && C == 4) {
        if (!hs && !sg.eio) return dispatch_scan_f<T, A, C, 2, false>(sg, k, block, st, ws);
      }
      return hs ? dispatch_scan_f<T, A, C, VF, true>(sg, k, block, st, ws)
                : dispatch_scan_f<T, A, C, VF, false>(sg, k, block, st, ws);
    }
  }
  return hs ? dispatch_scan_f<T, A, C, 1, true>(sg, k, block, st, ws)
            : dispatch_scan_f<T, A, C, 1, false>(sg, k, block, st, ws);
}

template <typename T, typename A>
int dispatch_scan(int C, bool vec, bool hs, const Sig& sg, int k, int block, hipStream_t st, Workspace ws) {
  switch (C) {
    case 1: return dispatch_scan_c<T, A, 1>(vec, hs, sg, k, block, st, ws);
    case 2: return dispatch_scan_c<T, A, 2>(vec, hs, sg, k, block, st, ws);
    case 3: return dispatch_scan_c<T, A, 3>(vec, hs, sg, k, block, st, ws);
    case 4: return dispatch_scan_c<T, A, 4>(vec, hs, sg, k, block, st, ws);
    case 5: return dispatch_scan_c<T, A, 5>(vec, hs, sg, k, block, st, ws);
    case 6: return dispatch_scan_c<T, A, 6>(vec, hs, sg, k, block, st, ws);
    case 7: return dispatch_scan_c<T, A, 7>(vec, hs, sg, k, block, st, ws);
    case 8: return dispatch_scan_c<T, A, 8>(vec, hs, sg, k, block, st, ws);
    default: return MAVG_ERR_UNSUPPORTED;
  }
}

// ---- direct LDS-tiled launch ---------------------------------------------------
template <typename T, typename A, int C, int F, int U = 1, int WG = kWG, int NT = 0>
int launch_direct(const Sig& sg, int k, hipStream_t st, int xcd_remap = kRemapGroup) {
  constexpr int TF = WG * F * U;
  constexpr int VE = F * C;
  const long long nframes = sg.nframes;
  DirectParams p{};
  p.in = sg.in;
  p.out = sg.out;
  p.hist = sg.hist;
  p.nframes = nframes;
  p.pre = sg.pre;
  p.eio = sg.eio;
  p.k = k;
  p.o = make_out_params(k);
  p.m = (k - 1 + F - 1) / F;
  p.off = p.m * F - (k - 1);
  p.xcd_remap = xcd_remap;
  const size_t lds = (((size_t)(p.m + U * WG) * VE * sizeof(T)) + 15) & ~(size_t)15;
  if (lds > kLdsBudget) return MAVG_ERR_UNSUPPORTED;
  const long long nblk = (nframes + TF - 1) / TF;
  if (nblk > 0x7fffffffLL) return MAVG_ERR_UNSUPPORTED;
  if (g_plan) {
    snprintf(g_plan->text, sizeof(g_plan->text), "direct<%s,acc=%s,C=%d,F=%d,U=%d,nt=%d> grid=%lld block=%d lds=%zu",
             type_name<T>(), type_name<A>(), C, F, U, NT, nblk, WG, lds);
    return MAVG_OK;
  }
  hipLaunchKernelGGL((direct_kernel<T, A, C, F, U, WG, NT>), dim3((unsigned)nblk), dim3(WG), lds, st, p);
  return hipGetLastError() == hipSuccess ? MAVG_OK : MAVG_ERR_HIP;
}

// The tuned direct launch: two units per lane, non-temporal tile, halo and
// output (2^28 fp32, k=7, in-process A/B, tools/tune/tune_scan.hip "dirnt":
// 0.835 of peak vs 0.814 for one unit per lane with the default policy;
// profiles/r02_tuning/r02_direct_nt/).  A reference block size keeps one unit
// per lane in a workgroup of that size.
constexpr int kNtDirect = kNtLoad | kNtHalo | kNtStore;
// A reference block size whose geometry does not fit the window's halo in LDS
// falls back to the tuned launch (as the scan dispatch does; mavg.h: "while
// the window's halo fits that workgroup's LDS").
template <typename T, typename A, int C, int F>
int launch_direct_block(const Sig& sg, int k, int block, hipStream_t st) {
  auto lds_fits = [&](int U, int WG) {
    const long long m = (k - 1 + F - 1) / F;
    return ((m + (long long)U * WG) * F * C * (long long)sizeof(T) + 15) / 16 * 16 <= (long long)kLdsBudget;
  };
  const int wg = block == 0 ? 0 : block_wg(block);
  if (wg != 0 && lds_fits(1, wg)) {
    switch (wg) {
      case 64: return launch_direct<T, A, C, F, 1, 64, kNtDirect>(sg, k, st);
      case 128: return launch_direct<T, A, C, F, 1, 128, kNtDirect>(sg, k, st);
      case 512: return launch_direct<T, A, C, F, 1, 512, kNtDirect>(sg, k, st);
      case 1024: return launch_direct<T, A, C, F, 1, 1024, kNtDirect>(sg, k, st);
      default: return launch_direct<T, A, C, F, 1, kWG, kNtDirect>(sg, k, st);
    }
  }
  return launch_direct<T, A, C, F, 2, kWG, kNtDirect>(sg, k, st);
}

// width: 16 (vload4), 8 (vload2) or 0 (one frame per lane); block: the
// reference's block size (0 = 256 threads)
template <typename T, typename A, int C>
int dispatch_direct_c(int width, const Sig& sg, int k, int block, hipStream_t st) {
  constexpr int FB = C * (int)sizeof(T);
  constexpr int F16 = (FB <= 16 && 16 % FB == 0) ? 16 / FB : 0;
  constexpr int F8 = (FB <= 8 && 8 % FB == 0) ? 8 / FB : 0;
  if constexpr (F16 > 0) {
    if (width == 16) return launch_direct_block<T, A, C, F16>(sg, k, block, st);
  }
  if constexpr (F8 > 0) {
    if (width >= 8) return launch_direct_block<T, A, C, F8>(sg, k, block, st);
  }
  return launch_direct_block<T, A, C, 1>(sg, k, block, st);
}

template <typename T, typename A>
int dispatch_direct(int C, int width, const Sig& sg, int k, int block, hipStream_t st) {
  switch (C) {
    case 1: return dispatch_direct_c<T, A, 1>(width, sg, k, block, st);
    case 2: return dispatch_direct_c<T, A, 2>(width, sg, k, block, st);
    case 3: return dispatch_direct_c<T, A, 3>(width, sg, k, block, st);
    case 4: return dispatch_direct_c<T, A, 4>(width, sg, k, block, st);
    case 5: return dispatch_direct_c<T, A, 5>(width, sg, k, block, st);
    case 6: return dispatch_direct_c<T, A, 6>(width, sg, k, block, st);
    case 7: return dispatch_direct_c<T, A, 7>(width, sg, k, block, st);
    case 8: return dispatch_direct_c<T, A, 8>(width, sg, k, block, st);
    default: return MAVG_ERR_UNSUPPORTED;
  }
}

// naive: one thread per sample, exactly `block` threads per workgroup (any
// multiple of 32 in [32, 1024], as the reference launches; 0 = 256)
template <typename T, typename A>
int launch_naive(const Sig& sg, int C, int k, int block, hipStream_t st) {
  const int wg = block == 0 ? kWG : block;
  const long long n = sg.nframes * C;
  const long long nblk = (n + wg - 1) / wg;
  if (nblk > 0x7fffffffLL) return MAVG_ERR_UNSUPPORTED;
  if (g_plan) {
    snprintf(g_plan->text, sizeof(g_plan->text), "naive<%s,acc=%s> grid=%lld block=%d", type_name<T>(),
             type_name<A>(), nblk, wg);
    return MAVG_OK;
  }
  hipLaunchKernelGGL((naive_kernel<T, A>), dim3((unsigned)nblk), dim3(wg), 0, st, static_cast<const T*>(sg.in),
                     static_cast<T*>(sg.out), static_cast<const T*>(sg.hist), sg.nframes, C, k, make_out_params(k));
  return hipGetLastError() == hipSuccess ? MAVG_OK : MAVG_ERR_HIP;
}

}  // namespace mavg
