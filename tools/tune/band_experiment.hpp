// band_experiment.hpp -- KEPT-OUT EXPERIMENT (round 3), not part of libmavg.
//
// The row-band scan for long windows: rows of k frames, so x[n-k] is the same
// LDS column one row up and every sample crosses the CU (M+1)/M times; the
// window sum in front of each row tile is the sum of S = k/T row-tile sums,
// all produced by the band's own S column workgroups (no look-ahead read, no
// chain).  Correct on MI355X (70 long-window parity tests incl. the
// forced-recompute schedule, profiles/r03_tuning/band/).  Slow: 0.48 of HBM
// peak against 0.71 for the look-ahead scan (2^30 fp32, k=44100; int16 stereo
// 0.44 vs 0.64).  The MAVG_BAND_TRACE phase trace (band_trace.py) shows why:
// every workgroup waits for the slowest of its band's 44 members to publish,
// 5.6 us after its own publish (median; int16 8.2 us), and the 36 KiB row stage
// allows ~3.3 workgroups per CU, so the 15 us lifetime cannot keep enough
// bytes in flight.  DESIGN.md "Tried this round".
//
// To rebuild it, include this file after mavg_launch.hpp in a tuning
// translation unit and call launch_band_scan<...>(...).
#pragma once

#include "../../digital_signal_processsing_amd/csrc/mavg_launch.hpp"

namespace mavg {

// ----------------------------------------------------------------------------
// Lay the signal out as rows of k frames: row j = frames [j*k, (j+1)*k).  Then
// x[n-k] is the frame in the same column one row up, and the window ending
// just before column s of row j is the tail of row j-1 from column s plus the
// head of row j before column s:
//     W[j*k + s*T - 1] = sum_{s' >= s} R(j-1, s') + sum_{s' < s} R(j, s')
// with R(j, s) the x-sum of the row tile (j, s) (T frames wide, the last
// column k - (S-1)*T).  A "band" is M consecutive output rows.  Workgroup
// (band b, column s) stages the M+1 row tiles (j-1 .. j+M-1 of column s) in
// LDS, publishes their sums R as tagged granules, reads the S sums of each
// window it needs from the band's other workgroups -- dispatched right
// beside it, so their records are the band's own loads, never a read ahead
// or a chain -- and scans d = x - x[n-k] row tile by row tile, x and x[n-k]
// at the same LDS offset of adjacent rows (no misaligned extraction).  Every
// sample crosses the CU (M+1)/M times.  Columns are padded to a multiple of 8
// workgroups, so column s always runs on the XCD of label s mod 8: the row a
// band re-reads (the previous band's last output row) is an L2 hit there.
//
// Determinism: R(j, s) is one fixed sum (lane l sums units u*64 + l over u,
// frames, then one DPP wave scan) whether its owner stages it from LDS or a
// waiting wave recomputes it from global memory after a bounded spin; the
// window sum adds the S records in a fixed lane order.  The window's own
// tiles only: no prefix differences, no error carried along the signal.
// ----------------------------------------------------------------------------
struct BandParams {
  const void* in;
  void* out;
  const void* hist;
  long long nframes;
  long long nbands;
  int k;
  int S;      // columns per row: ceil(k / T)
  int Sp;     // S padded to a multiple of 8 (XCD placement by column)
  int spin;   // polls of an unpublished record before recomputing it
  int pre;    // frames in front of `in` that are readable signal (load_elem)
  unsigned long long* rec;  // [nbands][M+1][S][C][NG] row-tile sums, zeroed before the launch
  void* stats;              // MAVG_AHEAD_STATS builds only: {recomputes, polls that waited}
  unsigned long long* trace;  // MAVG_BAND_TRACE tuning builds only: [grid][8] stamps (tools/tune/band_trace.py)
  OutParams o;
};

// MAVG_BAND_TRACE (tuning builds only): per workgroup, 100-MHz wall-clock
// stamps of wave 0's phases -- 0 start, 1 rows staged (barrier), 2 its row
// sums published, 3 first window sum read, 4 end; 5 = the XCD it ran on
#ifdef MAVG_BAND_TRACE
#define MAVG_BTRACE(slot, v) (p.trace[(unsigned long long)blockIdx.x * 8 + (slot)] = (unsigned long long)(v))
#define MAVG_BNOW() __builtin_amdgcn_s_memrealtime()
#else
#define MAVG_BTRACE(slot, v) ((void)0)
#define MAVG_BNOW() 0ull
#endif

// The sum of row tile (row j, column s) with one wave: lane l takes units
// u*64 + l (u < UL) that lie inside the column, frames and channels in order,
// then one DPP wave scan.  `stage` != nullptr: the units from the LDS row
// (owner); else from global memory (recompute), guarded at the signal's ends.
template <typename T, typename SA, int C, int F, int UL>
__device__ __forceinline__ void row_tile_sum(const T* stage, const T* __restrict__ in, const T* __restrict__ hist,
                                             long long j, int s, int T_, int wunits, int lane, const BandParams& p,
                                             SA (&r)[C]) {
  constexpr int VE = F * C;
  using IO = UnitIO<T, VE>;
  SA ls[C];
#pragma unroll
  for (int c = 0; c < C; ++c) ls[c] = (SA)0;
  const long long f0 = j * (long long)p.k + (long long)s * T_;
#pragma unroll
  for (int u = 0; u < UL; ++u) {
    const int q = u * 64 + lane;
    if (q < wunits) {
      Unit<T, VE> x;
      if (stage != nullptr) {
        x = IO::load(stage + q * VE);
      } else {
        const long long f = f0 + (long long)q * F;
#pragma unroll
        for (int fr = 0; fr < F; ++fr)
#pragma unroll
          for (int c = 0; c < C; ++c) x.e[fr * C + c] = load_elem(in, hist, f + fr, c, C, p.nframes, p.k, p.pre);
      }
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) ls[c] += to_acc<SA>(x.e[fr * C + c]);
    }
  }
#pragma unroll
  for (int c = 0; c < C; ++c) r[c] = readlane(wave_incl_scan(ls[c]), 63);
}

// NT: kNtLoad (rows no later band re-reads), kNtHalo (the re-read first row),
// kNtStore (outputs).  The band's last row keeps the default policy: the next
// band re-reads it from L2.
template <typename T, typename A, int C, int F, int UL, int M, int NT, int DV = 0>
__global__ __launch_bounds__(kWG) void band_scan_kernel(BandParams p) {
  constexpr int NW = kWG / 64;
  constexpr int VE = F * C;
  constexpr int TU = 64 * UL;        // units per row tile
  constexpr int T_ = TU * F;         // frames per row tile
  constexpr int NR = M + 1;          // staged rows: the row above the band + M output rows
  using IO = UnitIO<T, VE>;
  using U_t = Unit<T, VE>;
  using SA = typename ScanAcc<T, A>::type;
  constexpr int NGS = GranCount<SA>::n;
  constexpr bool kDma = IO::kVec && VE * (int)sizeof(T) == 16;

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* stage = reinterpret_cast<T*>(smem);  // [NR][TU] units

  const T* __restrict__ in = static_cast<const T*>(p.in);
  T* __restrict__ out = static_cast<T*>(p.out);
  const T* __restrict__ hist = static_cast<const T*>(p.hist);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wq = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int k = p.k;
  const long long nframes = p.nframes;

  const long long b = blockIdx.x / (unsigned)p.Sp;
  const int s = (int)(blockIdx.x % (unsigned)p.Sp);
  if (tid == 0) MAVG_BTRACE(0, MAVG_BNOW());
  if (s >= p.S) return;  // XCD padding column
  const int wframes = s == p.S - 1 ? k - (p.S - 1) * T_ : T_;
  const int wunits = wframes / F;  // k is a multiple of F (host)
  const long long j0 = b * M - 1;  // global row of staged row 0
  MAVG_DCHECK(b < p.nbands && wunits > 0 && wunits <= TU, "band tile", b, wunits);

  // ---- 1. stage the NR row tiles of column s (LDS-DMA where a whole
  //         64-unit segment lies inside the signal and the column) ----
#pragma unroll
  for (int i0 = 0; i0 < NR * UL; i0 += NW) {
    const int i = i0 + wq;
    if (i < NR * UL) {
      const int r = i / UL, u = i % UL;
      const long long fb = (j0 + r) * (long long)k + (long long)s * T_;  // first frame of the row tile
      const long long f = fb + (long long)(u * 64 + lane) * F;
      T* dst = stage + (r * TU + u * 64) * VE;
      const bool seg_fast = (u * 64 + 64 <= wunits) && fb + (long long)(u * 64) * F >= 0 &&
                            fb + (long long)(u * 64 + 64) * F <= nframes;
      if (kDma && seg_fast) {
        if constexpr (kDma) {
          const bool halo = r == 0, keep = r == NR - 1;
          if (halo ? (NT & kNtHalo) != 0 : (!keep && (NT & kNtLoad) != 0))
            glds16<true>(in + f * C, dst);
          else
            glds16<false>(in + f * C, dst);
        }
      } else {
        U_t x;
        if (seg_fast) {
          x = IO::load(in + f * C);
        } else {
#pragma unroll
          for (int fr = 0; fr < F; ++fr)
#pragma unroll
            for (int c = 0; c < C; ++c)
              x.e[fr * C + c] = u * 64 + lane < wunits ? load_elem(in, hist, f + fr, c, C, nframes, k, p.pre) : (T)0;
        }
        IO::store(dst + lane * VE, x);
      }
    }
  }
  __syncthreads();
  if (tid == 0) MAVG_BTRACE(1, MAVG_BNOW());

  // ---- 2. publish the row-tile sums of the staged rows (wave w: rows w, w+4, ..) ----
  gran_t* rec = (gran_t*)p.rec + (unsigned long long)b * NR * p.S * C * NGS;
#pragma unroll 1
  for (int r = wq; r < NR; r += NW) {
    SA rs[C];
    row_tile_sum<T, SA, C, F, UL>(stage + r * TU * VE, in, hist, j0 + r, s, T_, wunits, lane, p, rs);
    publish_record<SA, C>(rec, (long long)r * p.S + s, rs, lane);
  }
  if (tid == 0) MAVG_BTRACE(2, MAVG_BNOW());

  // ---- 3. output rows (wave w: rows 1+w, 1+w+4, ..): window sum from the
  //         band's records, then the row-tile scan of d = row r - row r-1 ----
#pragma unroll 1
  for (int r = 1 + wq; r < NR; r += NW) {
    const long long j = j0 + r;
    if (j * (long long)k + (long long)s * T_ >= nframes) break;  // past the end of the signal
    // W0 = sum_{s' >= s} R(r-1, s') + sum_{s' < s} R(r, s'): lane l takes
    // columns l, l+64, ... in order, one DPP wave scan
    A w0[C];
    {
      A acc[C];
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] = (A)0;
#pragma unroll 1
      for (int sb = 0; sb < p.S; sb += 64) {
        const int sc = sb + lane;
        const bool act = sc < p.S;
        const int rr = sc >= s ? r - 1 : r;
        const long long q = (long long)rr * p.S + (act ? sc : 0);
        unsigned long long g[C][NGS];
        bool ok = true;
#pragma unroll
        for (int c = 0; c < C; ++c)
#pragma unroll
          for (int h = 0; h < NGS; ++h) {
            g[c][h] = gran_load(rec + (q * C + c) * NGS + h);
            ok &= (g[c][h] >> 32) == 1ull;
          }
        ok |= !act;
#pragma unroll 1
        for (int it = 0, bo = 1; !__all(ok) && it < p.spin; ++it, bo = min(2 * bo, 16)) {
#ifdef MAVG_AHEAD_STATS
          if (lane == 0) atomicAdd(reinterpret_cast<unsigned int*>(p.stats) + 1, 1u);
#endif
          for (int z = 0; z < bo; ++z) __builtin_amdgcn_s_sleep(1);
          if (!ok) {
            ok = true;
#pragma unroll
            for (int c = 0; c < C; ++c)
#pragma unroll
              for (int h = 0; h < NGS; ++h) {
                g[c][h] = gran_load(rec + (q * C + c) * NGS + h);
                ok &= (g[c][h] >> 32) == 1ull;
              }
          }
        }
        unsigned long long miss = __ballot(!ok);
#pragma unroll 1
        while (miss != 0ull) {  // its owner has not published: recompute the row-tile sum, same bits
          const int l = __builtin_ctzll(miss);
          miss &= miss - 1ull;
          const int sl = sb + l;
          const int rl = sl >= s ? r - 1 : r;
          const int wl = sl == p.S - 1 ? (k - (p.S - 1) * T_) / F : TU;
          SA rs[C];
          row_tile_sum<T, SA, C, F, UL>(nullptr, in, hist, j0 + rl, sl, T_, wl, lane, p, rs);
          if (lane == l)
#pragma unroll
            for (int c = 0; c < C; ++c)
#pragma unroll
              for (int h = 0; h < NGS; ++h) g[c][h] = kGranTag | gran_word(rs[c], h);
#ifdef MAVG_AHEAD_STATS
          if (lane == 0) atomicAdd(reinterpret_cast<unsigned int*>(p.stats), 1u);
#endif
        }
        if (act)
#pragma unroll
          for (int c = 0; c < C; ++c) {
            uint32_t wd[NGS];
#pragma unroll
            for (int h = 0; h < NGS; ++h) wd[h] = (uint32_t)g[c][h];
            acc[c] += (A)gran_value<SA>(wd);
          }
      }
#pragma unroll
      for (int c = 0; c < C; ++c) w0[c] = readlane(wave_incl_scan(acc[c]), 63);
      if (tid == 0 && r == 1) MAVG_BTRACE(3, MAVG_BNOW());
    }
    // the row tile: 64-unit segments u, lane l owns unit u*64 + l (F frames)
    const long long fb = j * (long long)k + (long long)s * T_;
    const T* xr = stage + r * TU * VE;
    const T* kr = stage + (r - 1) * TU * VE;
    A carry[C];
#pragma unroll
    for (int c = 0; c < C; ++c) carry[c] = w0[c];
#pragma unroll
    for (int u = 0; u < UL; ++u) {
      const int q = u * 64 + lane;
      const U_t x = IO::load(xr + q * VE);
      const U_t xk = IO::load(kr + q * VE);
      SA v[F][C];
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) {
          const SA d = to_acc<SA>(x.e[fr * C + c]) - to_acc<SA>(xk.e[fr * C + c]);
          v[fr][c] = fr == 0 ? d : v[fr - 1][c] + d;
        }
      U_t y;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const SA incl = wave_incl_scan(v[F - 1][c]);
        const SA lx = incl - v[F - 1][c];
        const A base = carry[c] + (A)lx;
#pragma unroll
        for (int fr = 0; fr < F; ++fr) y.e[fr * C + c] = to_out<T, A, DV>(base + (A)v[fr][c], p.o);
        carry[c] += (A)readlane(incl, 63);
      }
      const long long f = fb + (long long)q * F;
      if (q < wunits) {
        if (f + F <= nframes) {
          IO::template store<(NT & kNtStore) != 0>(out + f * C, y);
        } else {
#pragma unroll
          for (int fr = 0; fr < F; ++fr)
            if (f + fr < nframes)
#pragma unroll
              for (int c = 0; c < C; ++c) out[(f + fr) * C + c] = y.e[fr * C + c];
        }
      }
    }
  }
  if (tid == 0) {
    MAVG_BTRACE(4, MAVG_BNOW());
#ifdef MAVG_BAND_TRACE
    MAVG_BTRACE(5, __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11)));
#endif
  }
}


// row-band scan (mavg_band.hpp): zero the record granules, then one launch of
// (bands x columns padded to a multiple of 8) workgroups.  Only for 16-B
// units whose rows start 16-B aligned (k a multiple of F) and at most 256
// columns; returns MAVG_ERR_UNSUPPORTED otherwise (the caller falls back).
// Workspace: one 8-B granule per (band, staged row, column, channel, 32-bit
// word of the tile sum), padded to 16 bytes, + 16 bytes of statistics.
template <typename T, typename A, int C, int F, int UL, int M>
struct BandLayout {
  using SA = typename ScanAcc<T, A>::type;
  static constexpr int T_ = 64 * UL * F;
  long long nbands;
  int S, Sp;
  size_t gran;
  BandLayout(long long nframes, int k) {
    S = (k + T_ - 1) / T_;
    Sp = (S + 7) / 8 * 8;
    const long long nrows = (nframes + k - 1) / k;
    nbands = (nrows + M - 1) / M;
    gran = (size_t)nbands * (M + 1) * S * C * GranCount<SA>::n;
  }
  size_t bytes() const { return (gran * 8 + 15) / 16 * 16 + 16 + trace_bytes(); }
#ifdef MAVG_BAND_TRACE
  size_t trace_bytes() const { return (size_t)nbands * Sp * 64; }
#else
  size_t trace_bytes() const { return 0; }
#endif
};
template <typename T, typename A, int C, int F, int UL, int M, int NT, int DV = 0>
int launch_band_scan(const Sig& sg, int k, hipStream_t st, Workspace ws) {
  constexpr int VE = F * C;
  constexpr int T_ = 64 * UL * F;
  if (VE * (int)sizeof(T) != 16 || k % F != 0 || sg.eio != 0) return MAVG_ERR_UNSUPPORTED;
  const BandLayout<T, A, C, F, UL, M> L(sg.nframes, k);
  if (L.S < 2 || L.S > 256) return MAVG_ERR_UNSUPPORTED;
  const long long grid = L.nbands * L.Sp;
  if (grid > 0x7fffffffLL) return MAVG_ERR_UNSUPPORTED;
  const size_t need = L.bytes();
  const size_t lds = (size_t)(M + 1) * 64 * UL * 16;
  int spin = kAheadSpin;
  {
    const int t = g_test_ahead_spin.load(std::memory_order_relaxed);
    if (t >= 0) spin = t;
  }
  if (g_plan) {
    snprintf(g_plan->text, sizeof(g_plan->text),
             "band_scan<%s,acc=%s,C=%d,F=%d,UL=%d,M=%d,nt=%d,dv=%d> grid=%lld block=%d lds=%zu tile_frames=%d "
             "columns=%d ws=%zu",
             type_name<T>(), type_name<A>(), C, F, UL, M, NT, DV, grid, kWG, lds, T_, L.S, need);
    g_plan->ws_bytes = need;
    return MAVG_OK;
  }
  if (ws.ptr == nullptr || ws.bytes < need) return MAVG_ERR_WORKSPACE;
  if ((reinterpret_cast<uintptr_t>(ws.ptr) & 15u) != 0) return MAVG_ERR_MISALIGNED;
  if (hipMemsetAsync(ws.ptr, 0, need, st) != hipSuccess) return MAVG_ERR_HIP;
  BandParams p{};
  p.in = sg.in;
  p.out = sg.out;
  p.hist = sg.hist;
  p.nframes = sg.nframes;
  p.nbands = L.nbands;
  p.k = k;
  p.S = L.S;
  p.Sp = L.Sp;
  p.spin = spin;
  p.pre = sg.pre;
  p.rec = static_cast<unsigned long long*>(ws.ptr);
  p.stats = static_cast<unsigned char*>(ws.ptr) + need - 16 - L.trace_bytes();
  p.trace = reinterpret_cast<unsigned long long*>(static_cast<unsigned char*>(ws.ptr) + need - L.trace_bytes());
  p.o = make_out_params(k);
  hipLaunchKernelGGL((band_scan_kernel<T, A, C, F, UL, M, NT, DV>), dim3((unsigned)grid), dim3(kWG), lds, st, p);
  return hipGetLastError() == hipSuccess ? MAVG_OK : MAVG_ERR_HIP;
}

// Long windows: the row-band scan where its geometry applies (16-B units,
// 16-B aligned rows, <= 256 columns), else the look-ahead scan.
template <typename T, typename A, int C, int F>
int dispatch_long(const Sig& sg, int k, hipStream_t st, Workspace ws) {
  constexpr int kNtB = kNtLoad | kNtHalo | kNtStore;
  if constexpr (F * C * (int)sizeof(T) == 16) {
    const int s = launch_band_scan<T, A, C, F, 4, 8, kNtB>(sg, k, st, ws);
    if (s != MAVG_ERR_UNSUPPORTED) return s;
  }
  return dispatch_ahead<T, A, C, F>(sg, k, st, ws);
}


}  // namespace mavg
