// wide_ab.hip -- in-process A/B of the wide-frame tile scan (mavg_wide.hpp)
// shapes against the library's own dispatch for multi-channel fp32 signals,
// interleaved rounds, one HIP-event pair per launch (bench.py's timing), the
// library's flat copy as the same-box ceiling.  Every variant's output is
// checked against the library's (|dy| <= 1e-6 |y|, fp64 sums in another order).
//
// build: make -C tools/tune wide_ab
// run:   tools/tune/wide_ab <log2n> <k> <C> [rounds] [dist] [f32|i16] [hs|self|selfhs|pair|xl]
// A copy of this file built against another tree's headers (round 5's wide_ab_prev / _cand /
// _r04) compares that tree's kernels with this library's: the library is linked -Bsymbolic, so
// its launches keep its own kernel code even where the template instances share a name.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <algorithm>
#include <string>
#include <vector>

#include "../../digital_signal_processsing_amd/csrc/mavg_launch.hpp"
#include "pair_ahead.hpp"

using namespace mavg;

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                                \
    }                                                                                         \
  } while (0)

struct Var {
  std::string name;
  std::function<int(hipStream_t)> run;
  std::vector<float> ms;
};

template <typename T, typename A, int C, int P, int U, int WG = 256, int DV = 0>
void add1(std::vector<Var>& vs, const Sig& sg, int k) {
  constexpr int kNtS = kNtSplit | kNtHalo | kNtStore;
  char name[64];
  snprintf(name, sizeof name, "wide P%d U%d %d ntS dv%d", P, U, WG, DV);
  vs.push_back({name, [=](hipStream_t s) { return launch_wide_tile<T, A, C, P, U, WG, kNtS, DV>(sg, k, s); }, {}});
}

template <typename T, typename A, int C, int Q, int WG, bool XG = false, int NT = kNtSplit | kNtHalo | kNtStore,
          bool IPOK = false, int XL = 0>
void addC(std::vector<Var>& vs, const Sig& sg, int k) {
  char name[64];
  snprintf(name, sizeof name, "chan Q%d %d nt%d xg%d%s%s", Q, WG, NT, (int)XG, XG && IPOK ? " ip" : "", XL ? " xl1" : "");
  vs.push_back({name, [=](hipStream_t s) { return launch_chan_tile<T, A, C, Q, WG, NT, 0, XG, IPOK, XL>(sg, k, s); }, {}});
}

// the round-3 unit kernels for the same C (tile_scan / ahead_scan, 32-B or 64-B units)
template <typename T, typename A, int C, int F>
void add_unit(std::vector<Var>& vs, const Sig& sg, int k, Workspace ws) {
  char name[64];
  snprintf(name, sizeof name, "r03 units F=%d", F);
  vs.push_back({name, [=](hipStream_t s) { return dispatch_scan_f<T, A, C, F, false>(sg, k, 0, s, ws); }, {}});
}

template <typename T, typename A, int C, int P, int UW, int WG, int F, int U, int DV = 0, bool XG = false>
void addA(std::vector<Var>& vs, const Sig& sg, int k, Workspace ws, int D = 1024) {
  constexpr int kNtA = kNtStore | kNtHalo;
  char name[80];
  snprintf(name, sizeof name, "wahead P%d U%d %d F%d U%d D%d dv%d xg%d", P, UW, WG, F, U, D, DV, (int)XG);
  vs.push_back({name, [=](hipStream_t s) {
                  return launch_wide_ahead<T, A, C, P, UW, WG, kNtA, DV, F, U, false, XG>(sg, k, s, ws, D);
                }, {}});
}

// the look-ahead scan with U units per lane (tile = U * WG * F frames), as dispatched otherwise
// self: self-published records (AheadParams::self) -- no phase A; every tile publishes its own
// record (its aggregate) as soon as its loads land and the carry reads the records after the
// in-tile scan (round 6: the aggregate-first form for the int16 long windows)
template <typename T, typename A, int C, int F, int U, bool RC, bool WREC, bool RUNS>
void addU(std::vector<Var>& vs, const Sig& sg, int k, Workspace ws, int D, size_t lds_floor = 0, bool self = false) {
  constexpr int kNtA = kNtStore | kNtHalo;
  char name[80];
  snprintf(name, sizeof name, "ahead U%d wrec=%d runs=%d D%d lds>=%zu%s", U, (int)WREC, (int)RUNS, D, lds_floor,
           self ? " self" : "");
  vs.push_back({name, [=](hipStream_t s) {
                  return launch_ahead_scan<T, A, C, F, U, kNtA, RC, true, WREC, 0, false, RUNS, 256>(sg, k, s, ws, D,
                                                                                                   self, lds_floor);
                }, {}});
}

// the wide look-ahead scan with the channel-per-lane in-tile scan (CH)
template <typename T, typename A, int C, int Q, int WG, int F, int U, bool XG = false, int MW = 0, int XL = 0>
void addAC(std::vector<Var>& vs, const Sig& sg, int k, Workspace ws, int D, bool self = false) {
  constexpr int kNtA = kNtStore | kNtHalo;
  char name[80];
  snprintf(name, sizeof name, "wahead chan Q%d %d F%d U%d D%d xg%d mw%d%s%s", Q, WG, F, U, D, (int)XG, MW,
           self ? " self" : "", XL == 2 ? " xl2" : (XL ? " xl1" : ""));
  vs.push_back({name, [=](hipStream_t s) {
                  return launch_wide_ahead<T, A, C, Q, 1, WG, kNtA, 0, F, U, true, XG, MW, XL>(sg, k, s, ws, D, self);
                }, {}});
}
// round 6: x of the halo-only channel-per-lane look-ahead as 16-B frame loads + quad transposes (XL)
// against the 4-B column loads, 16-B frames (fp32 4 channels, int16 8 channels)
template <typename T, typename A, int C>
void add_xl(std::vector<Var>& vs, const Sig& sg, int k, Workspace ws) {
  constexpr int kNtS = kNtSplit | kNtHalo | kNtStore;
  if (k <= 4096) {  // the halo-only channel tile's range (fp32 C = 4: k <= 3584, int16 C = 8: k <= 3072)
    if constexpr (sizeof(T) == 4 && C == 8) {
      addC<T, A, C, 32, 256, true>(vs, sg, k);
      addC<T, A, C, 32, 256, true, kNtS, false, 1>(vs, sg, k);
      addC<T, A, C, 32, 128, true>(vs, sg, k);
      addC<T, A, C, 32, 128, true, kNtS, false, 1>(vs, sg, k);
      addC<T, A, C, 16, 256, true, kNtS, false, 1>(vs, sg, k);
    } else if constexpr (sizeof(T) == 4 && C == 4) {
      addC<T, A, C, 32, 256, true, kNtS, true>(vs, sg, k);
      addC<T, A, C, 32, 256, true, kNtS, true, 1>(vs, sg, k);
      addC<T, A, C, 16, 256, true, kNtS, true>(vs, sg, k);
      addC<T, A, C, 16, 256, true, kNtS, true, 1>(vs, sg, k);
      addC<T, A, C, 16, 128, true, kNtS, true, 1>(vs, sg, k);
    } else if constexpr (sizeof(T) == 2 && C == 8) {
      addC<T, A, C, 32, 256, true>(vs, sg, k);
      addC<T, A, C, 32, 256, true, kNtS, false, 1>(vs, sg, k);
      addC<T, A, C, 16, 256, true>(vs, sg, k);
      addC<T, A, C, 16, 256, true, kNtS, false, 1>(vs, sg, k);
      addC<T, A, C, 16, 128, true, kNtS, false, 1>(vs, sg, k);
    }
    if (k < 2048) return;  // (the look-ahead shapes below: 2048-frame tiles)
  }
  if constexpr (sizeof(T) == 4 && C == 8) {
    if (k >= 1024) {
      addAC<T, A, C, 32, 256, 1, 4, true>(vs, sg, k, ws, 384);
      // round 6: self-published records in the one order every producer uses (fp32 too)
      addAC<T, A, C, 32, 256, 1, 4, true>(vs, sg, k, ws, 384, true);
      addAC<T, A, C, 32, 256, 1, 4, true, 0, 2>(vs, sg, k, ws, 384, true);
      if (getenv("WIDE_AB_SELF_ONLY")) return;
      for (int D : {256, 384, 512}) addAC<T, A, C, 32, 256, 1, 4, true, 0, 1>(vs, sg, k, ws, D);
      addAC<T, A, C, 16, 256, 1, 2, true, 0, 1>(vs, sg, k, ws, 768);
      addAC<T, A, C, 64, 256, 1, 8, true, 0, 1>(vs, sg, k, ws, 256);
    }
  } else if constexpr (sizeof(T) == 4 && C == 4) {
    // round 6: self-published records in the one order every producer uses (fp32 too)
    addAC<T, A, C, 32, 256, 1, 8, true, 0, 1>(vs, sg, k, ws, 384);
    addAC<T, A, C, 32, 256, 1, 8, true, 0, 2>(vs, sg, k, ws, 384, true);
    addAC<T, A, C, 32, 256, 1, 8, true>(vs, sg, k, ws, 384, true);
    addAC<T, A, C, 16, 256, 1, 4, true, 0, 2>(vs, sg, k, ws, 768, true);
    if (getenv("WIDE_AB_SELF_ONLY")) return;
    addAC<T, A, C, 16, 256, 1, 4, true>(vs, sg, k, ws, 768);
    addAC<T, A, C, 16, 256, 1, 4, true, 0, 1>(vs, sg, k, ws, 768);
    for (int D : {256, 320, 384, 448}) addAC<T, A, C, 32, 256, 1, 8, true, 0, 1>(vs, sg, k, ws, D);
    addAC<T, A, C, 32, 256, 1, 8, true, 4, 1>(vs, sg, k, ws, 384);
    addAC<T, A, C, 32, 128, 1, 8, true, 0, 1>(vs, sg, k, ws, 768);
    addP<T, A, C, 16, 256, 4, 1>(vs, sg, k, ws, 768);
    addP<T, A, C, 16, 256, 4, 1>(vs, sg, k, ws, 1024);
  } else if constexpr (sizeof(T) == 2 && C == 8) {
    addAC<T, A, C, 32, 256, 1, 8, true, 0, 1>(vs, sg, k, ws, 384);
    addAC<T, A, C, 32, 256, 1, 8, true, 0, 2>(vs, sg, k, ws, 384, true);
    if (getenv("WIDE_AB_SELF_ONLY")) return;
    addAC<T, A, C, 32, 256, 1, 8, true>(vs, sg, k, ws, 384);
    for (int D : {384, 512, 640}) addAC<T, A, C, 32, 256, 1, 8, true, 0, 1>(vs, sg, k, ws, D);
    addAC<T, A, C, 32, 512, 1, 8, true, 0, 2>(vs, sg, k, ws, 384, true);  // XL = 2: self-published
    addAC<T, A, C, 32, 256, 1, 8, true, 0, 2>(vs, sg, k, ws, 384, true);
    addAC<T, A, C, 32, 512, 1, 8, true>(vs, sg, k, ws, 384, true);
    addAC<T, A, C, 32, 512, 1, 8, true, 0, 1>(vs, sg, k, ws, 384);
    addP<T, A, C, 16, 256, 4, 1>(vs, sg, k, ws, 768);
  }
}

// the Hillis-Steele look-ahead (mono / stereo) at several look-ahead distances; per-wave records
// for mono as dispatched.  (Round 5 also measured the log-step scans rebuilt after the carry, RC:
// fewer registers, slower -- profiles/r05_tuning/hs/; the kernel no longer has that form.)
template <typename T, typename A, int C, int F, bool WREC, int U = 4>
void addH(std::vector<Var>& vs, const Sig& sg, int k, Workspace ws, int D) {
  constexpr int kNtA = kNtStore | kNtHalo;
  char name[80];
  snprintf(name, sizeof name, "hillis ahead U%d wrec=%d D%d", U, (int)WREC, D);
  vs.push_back({name, [=](hipStream_t s) {
                  return launch_ahead_scan<T, A, C, F, U, kNtA, false, true, WREC, 0, true, false, 256>(sg, k, s, ws, D);
                }, {}});
}
template <typename T, typename A, int C>
void add_hs(std::vector<Var>& vs, const Sig& sg, int k, Workspace ws) {
  constexpr int F = 16 / (C * (int)sizeof(T));
  for (int D : {384, 512, 768}) {
    if constexpr (C == 1) addH<T, A, C, F, true>(vs, sg, k, ws, D);
    else addH<T, A, C, F, false>(vs, sg, k, ws, D);
  }
  // half tiles: 76-82 VGPRs (fp32) instead of 120-126, 6 waves per SIMD instead of 4
  for (int D : {512, 768, 1024, 1536}) {
    addH<T, A, C, F, true, 2>(vs, sg, k, ws, D);
    addH<T, A, C, F, false, 2>(vs, sg, k, ws, D);
  }
}

// round 6: the look-ahead scan's record forms against each other at one shape -- look-ahead
// (phase A, D slots) or aggregate-first (self-published, no phase A), per-tile records, tiles of
// U units x WG threads
template <typename T, typename A, int C, int F, int U, int WG, bool HS = false, bool WREC = false>
void addS(std::vector<Var>& vs, const Sig& sg, int k, Workspace ws, int D, bool self) {
  constexpr bool RC = sizeof(T) == 4 && C == 1 && !HS;
  constexpr int kNtA = kNtStore | kNtHalo;
  char name[96];
  snprintf(name, sizeof name, "ahead%s U%d WG%d tile%d wrec=%d D%d%s", HS ? " hs" : "", U, WG, U * WG * F, (int)WREC,
           D, self ? " self" : "");
  vs.push_back({name, [=](hipStream_t s) {
                  return launch_ahead_scan<T, A, C, F, U, kNtA, RC, true, WREC, 0, HS, false, WG>(sg, k, s, ws, D, self);
                }, {}});
}
template <typename T, typename A, int C>
void add_self(std::vector<Var>& vs, const Sig& sg, int k, Workspace ws, bool hs) {
  constexpr int F = 16 / (C * (int)sizeof(T));
  if (!hs && k > 500000) {  // past the L2 reach (window-matched runs: D also sets the run length G)
    addS<T, A, C, F, 8, 256>(vs, sg, k, ws, 320, false);
    addS<T, A, C, F, 8, 256>(vs, sg, k, ws, 320, true);
    addS<T, A, C, F, 8, 256>(vs, sg, k, ws, 640, true);
    addS<T, A, C, F, 8, 256>(vs, sg, k, ws, 960, true);
    addS<T, A, C, F, 4, 256>(vs, sg, k, ws, 1024, true);
    return;
  }
  if (!hs) {
    addS<T, A, C, F, 4, 256>(vs, sg, k, ws, C == 1 ? 512 : 768, false);
    addS<T, A, C, F, 8, 256>(vs, sg, k, ws, 256, false);
    addS<T, A, C, F, 4, 256>(vs, sg, k, ws, 512, true);
    addS<T, A, C, F, 8, 256>(vs, sg, k, ws, 256, true);
    addS<T, A, C, F, 4, 512>(vs, sg, k, ws, 512, true);
    addS<T, A, C, F, 8, 512>(vs, sg, k, ws, 256, true);
  } else {
    addS<T, A, C, F, 4, 256, true, C == 1>(vs, sg, k, ws, 512, false);
    addS<T, A, C, F, 4, 256, true>(vs, sg, k, ws, 512, true);
    addS<T, A, C, F, 8, 256, true>(vs, sg, k, ws, 256, true);
    addS<T, A, C, F, 4, 512, true>(vs, sg, k, ws, 512, true);
  }
}

// round 6: the paired look-ahead (mavg_pair.hpp, two consecutive tiles per workgroup) against the
// one-tile halo-only channel-per-lane look-ahead at the same tile shape
template <typename T, typename A, int C, int Q, int WG, int U, int XL = 0>
void addP(std::vector<Var>& vs, const Sig& sg, int k, Workspace ws, int D) {
  constexpr int kNtA = kNtStore | kNtHalo;
  char name[80];
  snprintf(name, sizeof name, "pair chan Q%d %d U%d D%d%s", Q, WG, U, D, XL ? " xl1" : "");
  vs.push_back({name, [=](hipStream_t s) { return launch_pair_ahead<T, A, C, Q, WG, kNtA, 0, U, XL>(sg, k, s, ws, D); }, {}});
}
template <typename T, typename A, int C>
void add_pair(std::vector<Var>& vs, const Sig& sg, int k, Workspace ws) {
  if constexpr (sizeof(T) == 4 && C == 4) {
    addAC<T, A, C, 16, 256, 1, 4, true>(vs, sg, k, ws, 768);
    for (int D : {384, 768, 1024, 1536}) addP<T, A, C, 16, 256, 4>(vs, sg, k, ws, D);
  } else if constexpr (sizeof(T) == 4 && C == 8) {
    addAC<T, A, C, 32, 256, 1, 4, true>(vs, sg, k, ws, 384);
    addAC<T, A, C, 16, 256, 1, 2, true>(vs, sg, k, ws, 768);
    for (int D : {384, 768, 1536}) addP<T, A, C, 16, 256, 2>(vs, sg, k, ws, D);
  } else if constexpr (sizeof(T) == 2 && C == 8) {
    addAC<T, A, C, 32, 256, 1, 8, true>(vs, sg, k, ws, 384);
    addAC<T, A, C, 16, 256, 1, 4, true>(vs, sg, k, ws, 768);
    for (int D : {384, 768, 1536}) addP<T, A, C, 16, 256, 4>(vs, sg, k, ws, D);
  }
}

template <int C>
void add_wide_c(std::vector<Var>& vs, const Sig& sg, int k, Workspace ws);

template <int C>
void add_wide(std::vector<Var>& vs, const Sig& sg, int k, Workspace ws) {
  using T = float;
  using A = double;
  if constexpr (C == 1) {  // mono long windows: the wide look-ahead against the tuned look-ahead
    if (k > 384 * 4096) addU<T, A, C, 4, 4, true, false, true>(vs, sg, k, ws, 1024);
    else if (k > 63 * 4096) addU<T, A, C, 4, 4, true, false, false>(vs, sg, k, ws, 1024);
    else addU<T, A, C, 4, 4, true, true, false>(vs, sg, k, ws, 512);
    // 8192-frame tiles (the dispatch past the L2 reach): the look-ahead distance, and a footprint
    // cap through the LDS allocation (2 workgroups per CU instead of 3)
    for (int D : {128, 192, 256, 320, 384}) addU<T, A, C, 4, 8, true, false, false>(vs, sg, k, ws, D);
    for (int D : {160, 256, 320}) addU<T, A, C, 4, 8, true, false, false>(vs, sg, k, ws, D, 56 * 1024);
    // 4096-frame tiles (84-90 VGPRs, 5 waves per SIMD) against the 8192-frame ones (142, 3)
    for (int D : {384, 512, 640, 768}) addU<T, A, C, 4, 4, true, false, false>(vs, sg, k, ws, D);
  } else {
    add_wide_c<C>(vs, sg, k, ws);
  }
}

template <int C>
void add_wide_c(std::vector<Var>& vs, const Sig& sg, int k, Workspace ws) {
  using T = float;
  using A = double;
  if (k > 1024) {  // the look-ahead range: the unit look-ahead against the wide look-ahead shapes
    add_unit<T, A, C, C == 2 ? 2 : 1>(vs, sg, k, ws);
    if constexpr (C == 2) {
      addA<T, A, C, 8, 1, 256, 2, 4>(vs, sg, k, ws, 384);
      addA<T, A, C, 8, 1, 256, 2, 4>(vs, sg, k, ws, 512);
      addA<T, A, C, 8, 1, 256, 2, 4>(vs, sg, k, ws, 768);
    } else if constexpr (C == 4) {
      addA<T, A, C, 4, 1, 256, 1, 4>(vs, sg, k, ws, 512);
      // the halo-only (XG) channel-per-lane look-ahead
      addAC<T, A, C, 16, 256, 1, 4, true>(vs, sg, k, ws, 384);
      addAC<T, A, C, 16, 256, 1, 4, true>(vs, sg, k, ws, 512);
      addAC<T, A, C, 16, 256, 1, 4, true>(vs, sg, k, ws, 768);
      addAC<T, A, C, 16, 256, 1, 4, true>(vs, sg, k, ws, 1024);
      addAC<T, A, C, 16, 256, 1, 4, true, 5>(vs, sg, k, ws, 1024);
      addAC<T, A, C, 32, 256, 1, 8, true>(vs, sg, k, ws, 384);
      addAC<T, A, C, 32, 256, 1, 8, true>(vs, sg, k, ws, 512);
      addAC<T, A, C, 32, 256, 1, 8, true>(vs, sg, k, ws, 768);
      addAC<T, A, C, 32, 128, 1, 8, true>(vs, sg, k, ws, 512);
      addAC<T, A, C, 32, 128, 1, 8, true>(vs, sg, k, ws, 1024);
      // 4 workgroups per CU (<= 128 VGPRs) instead of 3 (142)
      addAC<T, A, C, 32, 256, 1, 8, true, 4>(vs, sg, k, ws, 384);
      addAC<T, A, C, 32, 256, 1, 8, true, 4>(vs, sg, k, ws, 512);
      addAC<T, A, C, 32, 256, 1, 8, true, 4>(vs, sg, k, ws, 768);
    } else {
      addAC<T, A, C, 32, 256, 1, 4>(vs, sg, k, ws, 512);
      // the halo-only (XG) channel-per-lane look-ahead
      addAC<T, A, C, 32, 256, 1, 4, true>(vs, sg, k, ws, 256);
      addAC<T, A, C, 32, 256, 1, 4, true>(vs, sg, k, ws, 384);
      addAC<T, A, C, 32, 256, 1, 4, true>(vs, sg, k, ws, 512);
      addAC<T, A, C, 32, 256, 1, 4, true>(vs, sg, k, ws, 768);
      addAC<T, A, C, 32, 128, 1, 4, true>(vs, sg, k, ws, 512);
      addAC<T, A, C, 16, 256, 1, 2, true>(vs, sg, k, ws, 512);
    }
    if (k > 4096) return;
  }
  if constexpr (C == 2) {
    add_unit<T, A, C, 2>(vs, sg, k, ws);
    add1<T, A, C, 8, 1>(vs, sg, k);
    add1<T, A, C, 8, 2>(vs, sg, k);
    add1<T, A, C, 16, 1>(vs, sg, k);
    add1<T, A, C, 16, 1, 128>(vs, sg, k);
  } else if constexpr (C == 4) {
    add1<T, A, C, 8, 1>(vs, sg, k);
    addC<T, A, C, 16, 256, true>(vs, sg, k);
    addC<T, A, C, 32, 256, true>(vs, sg, k);
    addC<T, A, C, 32, 256, true, kNtSplit | kNtHalo | kNtStore, true>(vs, sg, k);
    addC<T, A, C, 16, 128, true>(vs, sg, k);
  } else {
    addC<T, A, C, 32, 256>(vs, sg, k);
    addC<T, A, C, 32, 256, true>(vs, sg, k);
    addC<T, A, C, 32, 256, true, kNtSplit | kNtHalo | kNtStore, true>(vs, sg, k);
    addC<T, A, C, 32, 128, true>(vs, sg, k);
    addC<T, A, C, 16, 128, true>(vs, sg, k);
  }
}

// int16 (the reference's PCM data path): int32 accumulators (k <= 65535)
template <int C>
void add_wide_i16(std::vector<Var>& vs, const Sig& sg, int k, Workspace ws) {
  using T = int16_t;
  using A = int32_t;
  constexpr int VF = 16 / (2 * C);
  add_unit<T, A, C, VF>(vs, sg, k, ws);
  if (k > 8192 || (C == 8 && k > 3072)) {  // the look-ahead range (8 channels: past the chan tile)
    if constexpr (C == 1) {  // mono: per-wave records, D = 512 (the library's dispatch)
      addU<T, A, C, 8, 4, false, true, false>(vs, sg, k, ws, 512);
      // aggregate-first (self-published records) against the look-ahead
      addU<T, A, C, 8, 4, false, true, false>(vs, sg, k, ws, 512, 0, true);
      addU<T, A, C, 8, 4, false, false, false>(vs, sg, k, ws, 512, 0, true);
      addU<T, A, C, 8, 8, false, false, false>(vs, sg, k, ws, 256, 0, true);
      addU<T, A, C, 8, 2, false, true, false>(vs, sg, k, ws, 512, 0, true);
      addU<T, A, C, 8, 4, false, true, false>(vs, sg, k, ws, 384);
      addU<T, A, C, 8, 8, false, false, false>(vs, sg, k, ws, 256);
      addU<T, A, C, 8, 8, false, false, false>(vs, sg, k, ws, 192);
    } else if constexpr (C == 2) {
      addU<T, A, C, 4, 8, false, false, false>(vs, sg, k, ws, 256);
      // aggregate-first (self-published records) against the look-ahead
      addU<T, A, C, 4, 8, false, false, false>(vs, sg, k, ws, 256, 0, true);
      addU<T, A, C, 4, 4, false, false, false>(vs, sg, k, ws, 512, 0, true);
      addU<T, A, C, 4, 4, false, true, false>(vs, sg, k, ws, 512, 0, true);
      addU<T, A, C, 4, 4, true, false, false>(vs, sg, k, ws, 768);   // recompute-from-registers (RC)
      addU<T, A, C, 4, 8, true, false, false>(vs, sg, k, ws, 256);
      addU<T, A, C, 4, 4, false, true, false>(vs, sg, k, ws, 512);   // per-wave records for stereo
      addU<T, A, C, 4, 4, false, true, false>(vs, sg, k, ws, 384);
      addU<T, A, C, 4, 8, false, true, false>(vs, sg, k, ws, 192);
      addU<T, A, C, 4, 8, false, true, false>(vs, sg, k, ws, 128);
    } else if constexpr (C == 4) {
      addA<T, A, C, 8, 1, 256, 2, 4>(vs, sg, k, ws, 384);
      addA<T, A, C, 8, 1, 256, 2, 4>(vs, sg, k, ws, 512);
      addA<T, A, C, 8, 1, 256, 2, 4>(vs, sg, k, ws, 768);
    } else {
      addA<T, A, C, 4, 1, 256, 1, 4>(vs, sg, k, ws, 1024);
      // the halo-only channel-per-lane look-ahead with a dword column (2 channels) per lane
      addAC<T, A, C, 32, 256, 1, 8, true>(vs, sg, k, ws, 256);
      addAC<T, A, C, 32, 256, 1, 8, true>(vs, sg, k, ws, 384);
      addAC<T, A, C, 32, 256, 1, 8, true>(vs, sg, k, ws, 512);
      addAC<T, A, C, 16, 256, 1, 4, true>(vs, sg, k, ws, 512);
      addAC<T, A, C, 16, 256, 1, 4, true>(vs, sg, k, ws, 768);
      // aggregate-first (self-published records from the registers) against the look-ahead
      addAC<T, A, C, 32, 256, 1, 8, true>(vs, sg, k, ws, 384, true);
      // 4096-frame tiles (a window of 11 instead of 21): 512 threads, or 64 frames per lane
      addAC<T, A, C, 32, 512, 1, 8, true>(vs, sg, k, ws, 384, true);
      addAC<T, A, C, 32, 512, 1, 8, true>(vs, sg, k, ws, 384);
      addAC<T, A, C, 64, 256, 1, 16, true>(vs, sg, k, ws, 384, true);
      addAC<T, A, C, 64, 256, 1, 16, true>(vs, sg, k, ws, 384);
    }
    return;
  }
  if constexpr (C == 2) {
    add1<T, A, C, 16, 1, 256, 0>(vs, sg, k);
    add1<T, A, C, 16, 1, 256, 1>(vs, sg, k);
  } else if constexpr (C == 4) {
    add1<T, A, C, 8, 1, 256, 0>(vs, sg, k);
    add1<T, A, C, 8, 1, 256, 1>(vs, sg, k);  // the magic-multiply division
    add1<T, A, C, 16, 1, 256, 0>(vs, sg, k);
    add1<T, A, C, 8, 2, 256, 0>(vs, sg, k);
    add1<T, A, C, 8, 1, 512, 0>(vs, sg, k);  // 4096-frame tiles: a quarter of the tile's halo
    // round 6: 1024-frame tiles (128 threads; 32-B chunks are not a chunk shape)
    add1<T, A, C, 8, 1, 128, 0>(vs, sg, k);
    if (getenv("WIDE_AB_TILES_ONLY")) return;
  } else if constexpr (C == 8) {
    add1<T, A, C, 8, 1, 256, 0>(vs, sg, k);
    add1<T, A, C, 8, 1, 256, 1>(vs, sg, k);  // the magic-multiply division
    add1<T, A, C, 4, 2, 256, 0>(vs, sg, k);
    // round 6: 1024-frame tiles (half the stage: 5 workgroups per CU by LDS)
    add1<T, A, C, 4, 1, 256, 0>(vs, sg, k);
    add1<T, A, C, 8, 1, 128, 0>(vs, sg, k);
    if (getenv("WIDE_AB_TILES_ONLY")) return;
    // the halo-only channel-per-lane look-ahead (82 VGPRs) at tile-scan windows too
    addAC<T, A, C, 16, 256, 1, 4, true>(vs, sg, k, ws, 384);
    addAC<T, A, C, 16, 256, 1, 4, true>(vs, sg, k, ws, 512);
    addAC<T, A, C, 32, 256, 1, 8, true>(vs, sg, k, ws, 384);
    // the channel-per-lane tile with two channels (a dword column) per lane
    addC<T, A, C, 32, 256>(vs, sg, k);
    addC<T, A, C, 16, 256>(vs, sg, k);
    addC<T, A, C, 16, 128>(vs, sg, k);
    addC<T, A, C, 16, 256, true>(vs, sg, k);
    addC<T, A, C, 32, 256, true>(vs, sg, k);
    addC<T, A, C, 32, 256, true, kNtSplit | kNtHalo | kNtStore, true>(vs, sg, k);
    addC<T, A, C, 16, 128, true>(vs, sg, k);
  }
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 30;
  const int k = argc > 2 ? atoi(argv[2]) : 1024;
  const int C = argc > 3 ? atoi(argv[3]) : 4;
  const int rounds = argc > 4 ? atoi(argv[4]) : 6;
  const int dist = argc > 5 ? atoi(argv[5]) : 1;
  const bool i16 = argc > 6 && std::string(argv[6]) == "i16";
  const bool hs = argc > 7 && std::string(argv[7]) == "hs";  // the Hillis-Steele look-ahead forms
  // "self" / "selfhs": the record forms of the look-ahead scan (add_self), Blelloch / Hillis-Steele
  const bool selfab = argc > 7 && (std::string(argv[7]) == "self" || std::string(argv[7]) == "selfhs");
  const bool selfhs = argc > 7 && std::string(argv[7]) == "selfhs";
  const bool pairab = argc > 7 && std::string(argv[7]) == "pair";  // the paired look-ahead (add_pair)
  const bool xlab = argc > 7 && std::string(argv[7]) == "xl";  // 16-B frame loads (add_xl)
  const int algo = hs || selfhs ? MAVG_ALGO_HILLIS : MAVG_ALGO_BLELLOCH;
  const int dt = i16 ? MAVG_I16 : MAVG_F32;
  const int eb = i16 ? 2 : 4;
  const int steps = 10;
  const long long n = 1LL << lg;
  void *x, *y, *yref;
  CK(hipMalloc(&x, n * eb));
  CK(hipMalloc(&y, n * eb));
  CK(hipMalloc(&yref, n * eb));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  if (mavg_fill_synthetic(x, n, dt, 0x5EED, 0, i16 ? 0 : dist, st) != MAVG_OK) return 1;
  size_t wsb = 0;
  mavg_workspace_bytes(n, C, k, dt, algo, 0, &wsb);
  const size_t ws2 = std::max<size_t>(wsb, 256u << 20);  // also the r03 unit kernels' look-ahead records
  void* ws = nullptr;
  CK(hipMalloc(&ws, ws2));
  char plan[256];
  mavg_plan(n, C, k, dt, algo, 0, plan, sizeof plan);

  const Sig sg{x, y, nullptr, n / C};
  std::vector<Var> vs;
  vs.push_back({std::string("lib: ") + plan, [=](hipStream_t s) {
                  return mavg_run(x, y, n, C, k, dt, algo, 0, nullptr, ws, wsb, s);
                }, {}});
  vs.push_back({"copy", [=](hipStream_t s) { return mavg_stream_copy(x, y, n * eb, s); }, {}});
  const Workspace w2{ws, ws2};
  if (xlab) {
    switch (C * (i16 ? -1 : 1)) {
      case 4: add_xl<float, double, 4>(vs, sg, k, w2); break;
      case 8: add_xl<float, double, 8>(vs, sg, k, w2); break;
      case -8: add_xl<int16_t, int32_t, 8>(vs, sg, k, w2); break;
      default: fprintf(stderr, "xl: f32 C=4/8, i16 C=8\n"); return 1;
    }
  } else if (pairab) {
    switch (C * (i16 ? -1 : 1)) {
      case 4: add_pair<float, double, 4>(vs, sg, k, w2); break;
      case 8: add_pair<float, double, 8>(vs, sg, k, w2); break;
      case -8: add_pair<int16_t, int32_t, 8>(vs, sg, k, w2); break;
      default: fprintf(stderr, "pair: f32 C=4/8, i16 C=8\n"); return 1;
    }
  } else if (selfab) {
    switch (C * (i16 ? -1 : 1)) {
      case 1: add_self<float, double, 1>(vs, sg, k, w2, selfhs); break;
      case 2: add_self<float, double, 2>(vs, sg, k, w2, selfhs); break;
      case -1: add_self<int16_t, int32_t, 1>(vs, sg, k, w2, selfhs); break;
      case -2: add_self<int16_t, int32_t, 2>(vs, sg, k, w2, selfhs); break;
      case 4: add_self<float, double, 4>(vs, sg, k, w2, selfhs); break;
      case -4: add_self<int16_t, int32_t, 4>(vs, sg, k, w2, selfhs); break;
      case -8: add_self<int16_t, int32_t, 8>(vs, sg, k, w2, selfhs); break;
      default: fprintf(stderr, "self: f32 C=1/2/4, i16 C=1/2/4/8\n"); return 1;
    }
  } else if (hs) {
    if (C == 1 && !i16) add_hs<float, double, 1>(vs, sg, k, w2);
    else if (C == 2 && i16) add_hs<int16_t, int32_t, 2>(vs, sg, k, w2);
    else if (C == 1 && i16) add_hs<int16_t, int32_t, 1>(vs, sg, k, w2);
    else { fprintf(stderr, "hs: f32 mono, i16 mono or stereo\n"); return 1; }
  } else
  switch (C * (i16 ? -1 : 1)) {
    case 1: add_wide<1>(vs, sg, k, w2); break;
    case 2: add_wide<2>(vs, sg, k, w2); break;
    case 4: add_wide<4>(vs, sg, k, w2); break;
    case 8: add_wide<8>(vs, sg, k, w2); break;
    case -1: add_wide_i16<1>(vs, sg, k, w2); break;
    case -2: add_wide_i16<2>(vs, sg, k, w2); break;
    case -4: add_wide_i16<4>(vs, sg, k, w2); break;
    case -8: add_wide_i16<8>(vs, sg, k, w2); break;
    default: fprintf(stderr, "C must be 1, 2, 4 or 8\n"); return 1;
  }
  // the library's launch once more, last in the list (the first entry's position in the interleaved
  // order is not neutral: it follows the copy in every forward round)
  vs.push_back({"lib (last)", vs[0].run, {}});
  // WIDE_AB_LIST: the variants' indices; WIDE_AB_ONLY=<i>: variant i alone, 1 + 10 launches and no
  // check -- every dispatch of such a run apart from the input fill and the workspace memsets is
  // variant i's, so one rocprofv3 --pmc pass measures that variant (tools/gpu/r05_footprint_pmc.sh)
  if (getenv("WIDE_AB_LIST")) {
    for (size_t v = 0; v < vs.size(); ++v) printf("%zu\t%s\n", v, vs[v].name.c_str());
    return 0;
  }
  if (const char* only = getenv("WIDE_AB_ONLY")) {
    const int vi = atoi(only);
    if (vi < 0 || vi >= (int)vs.size()) {
      fprintf(stderr, "WIDE_AB_ONLY=%d: %zu variants\n", vi, vs.size());
      return 1;
    }
    for (int i = 0; i < 1 + steps; ++i)
      if (vs[vi].run(st) != MAVG_OK) return 1;
    CK(hipStreamSynchronize(st));
    printf("%d\t%s\n", vi, vs[vi].name.c_str());
    return 0;
  }
  // reference output: the library
  if (vs[0].run(st) != MAVG_OK) return 1;
  CK(hipMemcpyAsync(yref, y, n * eb, hipMemcpyDeviceToDevice, st));
  CK(hipStreamSynchronize(st));
  std::vector<float> href(n), h(n);
  std::vector<int16_t> sref(i16 ? n : 0), sh(i16 ? n : 0);
  if (i16) CK(hipMemcpy(sref.data(), yref, n * eb, hipMemcpyDeviceToHost));
  else CK(hipMemcpy(href.data(), yref, n * eb, hipMemcpyDeviceToHost));
  for (size_t v = 2; v < vs.size(); ++v) {
    CK(hipMemsetAsync(y, 0xff, n * eb, st));
    const int rc = vs[v].run(st);
    CK(hipStreamSynchronize(st));
    if (rc != MAVG_OK) {
      printf("%-40s rc=%d (skipped)\n", vs[v].name.c_str(), rc);
      vs[v].run = nullptr;
      continue;
    }
    long long bad = 0;
    double worst = 0;
    if (i16) {  // bit-exact
      CK(hipMemcpy(sh.data(), y, n * eb, hipMemcpyDeviceToHost));
      for (long long i = 0; i < n; ++i) bad += sh[i] != sref[i];
    } else {
      CK(hipMemcpy(h.data(), y, n * eb, hipMemcpyDeviceToHost));
    }
    for (long long i = 0; !i16 && i < n; ++i) {
      const double r = href[i], d = std::fabs((double)h[i] - r);
      const double rel = d / std::max(std::fabs(r), 1e-30);
      if (!(d <= 1e-6 * std::fabs(r) || d == 0.0)) {
        if (bad < 5) printf("  mismatch %s at %lld: %.9g vs %.9g\n", vs[v].name.c_str(), i, h[i], r);
        ++bad;
      }
      if (d != 0.0 && rel > worst) worst = rel;
    }
    g_plan = nullptr;
    printf("%-40s check: %lld bad, max rel %.3g\n", vs[v].name.c_str(), bad, worst);
    if (bad) vs[v].run = nullptr;
  }
  hipEvent_t e0[steps], e1[steps];
  for (int i = 0; i < steps; ++i) {
    CK(hipEventCreate(&e0[i]));
    CK(hipEventCreate(&e1[i]));
  }
  for (int r = 0; r < rounds; ++r) {
    for (size_t vi = 0; vi < vs.size(); ++vi) {
      Var& v = vs[(r & 1) ? vs.size() - 1 - vi : vi];
      if (!v.run) continue;
      v.run(st);  // warm
      for (int i = 0; i < steps; ++i) {
        CK(hipEventRecord(e0[i], st));
        v.run(st);
        CK(hipEventRecord(e1[i], st));
      }
      CK(hipStreamSynchronize(st));
      for (int i = 0; i < steps; ++i) {
        float ms;
        CK(hipEventElapsedTime(&ms, e0[i], e1[i]));
        v.ms.push_back(ms);
      }
    }
  }
  printf("n=2^%d k=%d C=%d %s rounds=%d dist=%d (fraction of 8 TB/s, mean of per-launch events)\n", lg, k, C,
         i16 ? "i16" : "f32", rounds, dist);
  for (auto& v : vs) {
    if (v.ms.empty()) continue;
    double m = 0;
    for (float t : v.ms) m += t;
    m /= v.ms.size();
    std::vector<float> s = v.ms;
    std::sort(s.begin(), s.end());
    const double md = s[s.size() / 2];
    printf("%-72s mean %.4f ms  %.4f   median %.4f\n", v.name.c_str(), m, 2.0 * eb * n / (m * 1e-3) / 8e12,
           2.0 * eb * n / (md * 1e-3) / 8e12);
  }
  return 0;
}
