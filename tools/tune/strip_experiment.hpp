// strip_experiment.hpp -- KEPT-OUT EXPERIMENT (round 2, not built into libmavg):
// the strip scan, long windows with every sample read through the CU once.
// Correct (20 GPU parity cases against the oracle, bitwise equal under forced
// record recompute and 1/2/3-row blocks: profiles/r02_tuning/r02_strip/) but
// 0.25-0.39 of HBM peak against the look-ahead scan's 0.60-0.69 in the same
// process -- its in-flight bytes are one row tile per workgroup (DESIGN.md,
// "Tried this round and not kept").  It was launched with WG + 64 threads, the
// grid sized to the resident capacity (hipOccupancyMaxActiveBlocksPerMultiprocessor),
// the granules zeroed before each launch like the look-ahead scan's.
#pragma once

#include "../../digital_signal_processsing_amd/csrc/mavg_lookback.hpp"

namespace mavg {

// ----------------------------------------------------------------------------
// strip scan: the signal as rows of k frames
//
// Lay the signal out as a matrix of rows of k frames: row j holds frames
// [j*k, (j+1)*k), column c frame j*k + c.  Then x[n-k] is the SAME column of
// the row above, and with W the window sum
//     W_j[c] = W_j[c0-1] + sum_{c0 <= c' <= c} (x_j[c'] - x_{j-1}[c'])
// so a workgroup that owns the column strip [c0, c1) and walks down the rows
// keeps the row above in registers: d = x - x[n-k] needs no second read of
// the signal (the look-ahead scan reads every x[n-k] again from L2, which
// bounds it at 0.63-0.74 of HBM peak).
//
// The carry W_j[c0-1] is a window of k frames: row j-1's columns [c0, k) and
// row j's columns [0, c0) -- exactly one tile of every strip, so
//     W_j[c0-1] = sum_{s' < s} Tsum(j, s') + sum_{s' >= s} Tsum(j-1, s')
// with Tsum(j, s') the sum of strip s' in row j.  Every workgroup publishes the
// per-wave shares of its tiles' sums as tagged granules (mavg_lookback.hpp:
// {tag, 32-bit word}, agent-scope stores, the data is the flag) one row AHEAD
// of its scan -- the row it has just prefetched -- so its siblings find them
// when they reach that row.  No record depends on another record: there is no
// chain to wait along.
//
// Geometry: S strips of <= U*WG units cover a row; R consecutive rows form a
// row-block; workgroup (block b, strip s) walks rows [b*R, (b+1)*R).  The S
// strips of a block are dispatched adjacently on one XCD (blockIdx & 7), so
// their records stay in that XCD's L2.  The host sizes the grid to the
// resident capacity (all workgroups co-resident, siblings in step); a
// workgroup's first row reads the row above its block (1/R extra traffic).
//
// Progress never depends on scheduling: a granule still untagged after a
// bounded number of polls is recomputed by the waiting wave from the input,
// with the producer's lane mapping and order of operations -- bitwise the same
// value, so the same output.  Records are indexed by global row, so the two
// blocks that publish a block boundary's row store identical bits.  The
// granules are zeroed before every launch.
//
// Per step (one row) a scan wave issues the loads of row j+3, publishes its
// share of row j+2 (loaded a step ago), scans d = x_j - x_{j-1} (in-lane, DPP
// wave scan, segment totals through LDS, one barrier) and writes row j; a
// separate carry wave polls the records of row j (its own vmcnt, so a poll
// never waits behind the scan's loads and stores) and hands W_j[c0-1] over in
// LDS at that barrier.  The five row buffers rotate by unrolling the walk five
// times (a register copy of an in-flight load would wait for it).
// ----------------------------------------------------------------------------
struct StripParams {
  const void* in;
  void* out;
  const void* hist;
  long long nframes;
  long long nrows;  // rows holding output frames: ceil(nframes / k)
  int k;            // frames per row (the window)
  int pre;          // frames in front of `in` that are readable signal (load_elem)
  int ku;           // units per row (k / F)
  int wu;           // units per strip (<= U * WG); the last strip may be narrower
  int nstrips;      // S
  int rows;         // R, rows per row-block
  int spin;         // polls of an untagged granule before recomputing it
  unsigned long long* gran;  // [nrows + 1][S][NW][C][NG] granules, zeroed before the launch
  OutParams o;
};

// WG compute threads (NW waves) + one carry wave
template <typename T, typename A, int C, int F, int U, int WG, int NT, int DV>
__global__ __launch_bounds__(WG + 64) void strip_scan_kernel(StripParams p) {
  constexpr int NW = WG / 64;
  constexpr int VE = F * C;
  constexpr int NSEG = U * NW;
  using IO = UnitIO<T, VE>;
  using U_t = Unit<T, VE>;
  using SA = typename ScanAcc<T, A>::type;
  constexpr int NG = GranCount<SA>::n;
  static_assert(NSEG <= 64, "segment totals are scanned across one wave");
  __shared__ SA tot[2][NSEG * C];
  __shared__ A cbuf[2][C];

  const T* __restrict__ in = static_cast<const T*>(p.in);
  T* __restrict__ out = static_cast<T*>(p.out);
  const T* __restrict__ hist = static_cast<const T*>(p.hist);
  gran_t* gran = (gran_t*)p.gran;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int wq = __builtin_amdgcn_readfirstlane(w);
  const int k = p.k;
  const int pre = p.pre;
  const long long nframes = p.nframes;
  const int S = p.nstrips;

  // (block, strip): the S strips of a block adjacent in dispatch order on XCD blockIdx & 7
  const unsigned xcd = blockIdx.x & 7u, i = blockIdx.x >> 3;
  const unsigned bl = i / (unsigned)S;
  const int s = (int)(i - bl * (unsigned)S);
  const long long j0 = ((long long)bl * 8 + xcd) * p.rows;
  if (j0 >= p.nrows) return;
  const int R = (int)(p.nrows - j0 < (long long)p.rows ? p.nrows - j0 : (long long)p.rows);
  const int c0 = s * p.wu;                                  // first unit of the strip in a row
  const int wcnt = p.ku - c0 < p.wu ? p.ku - c0 : p.wu;     // units in this strip

  auto tile_fast = [&](long long j, int cc0, int cnt) {
    return j >= 0 && j * k + (long long)(cc0 + cnt) * F <= nframes;
  };
  // Lane unit idx of tile (row j, strip at cc0 of cnt units).  Fast tiles load
  // every lane's unit unconditionally (lanes past the strip re-read its last
  // unit: no per-lane branch, so no wait at a join); those lanes only ever
  // feed scan positions after the strip's outputs, and the records mask them.
  auto load_tile_units = [&](long long j, int cc0, int cnt, int lane0, U_t (&v)[U]) {
    if (tile_fast(j, cc0, cnt)) {
      const T* base = in + (j * k + (long long)cc0 * F) * C;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int idx = u * WG + lane0;
        v[u] = IO::template load<(NT & kNtLoad) != 0>(base + (long long)(idx < cnt ? idx : cnt - 1) * VE);
      }
    } else {  // edge tiles (guarded); unrolled: a dynamic index would put v in scratch
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long f = j * k + (long long)(cc0 + u * WG + lane0) * F;
#pragma unroll
        for (int fr = 0; fr < F; ++fr)
#pragma unroll
          for (int c = 0; c < C; ++c) v[u].e[fr * C + c] = load_elem(in, hist, f + fr, c, C, nframes, k, pre);
      }
    }
  };
  // one wave's share of a tile's sum: lanes in order of units, masked to the strip
  auto share_sum = [&](const U_t (&v)[U], int cnt, int lane0, SA (&r)[C]) {
    SA ls[C];
#pragma unroll
    for (int c = 0; c < C; ++c) ls[c] = (SA)0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool on = u * WG + lane0 < cnt;
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) ls[c] += on ? to_acc<SA>(v[u].e[fr * C + c]) : (SA)0;
    }
#pragma unroll
    for (int c = 0; c < C; ++c) r[c] = readlane(wave_incl_scan(ls[c]), 63);
  };
  // record of (row j, strip ss, wave wv): granules at ((j + 1) * S + ss) * NW + wv
  auto rec_index = [&](long long j, int ss, int wv) { return ((j + 1) * S + ss) * NW + wv; };

  if (w == NW) {
    // ---- the carry wave: W_j[c0-1] for every row, one row ahead of the scan ----
    // (its own wave, so its polls never wait behind the scan's loads and stores)
    auto recompute = [&](long long j, int ss, int wv, SA (&r)[C]) {
      const int cc0 = ss * p.wu;
      const int cnt = p.ku - cc0 < p.wu ? p.ku - cc0 : p.wu;
      U_t v[U];
      load_tile_units(j, cc0, cnt, wv * 64 + lane, v);
      share_sum(v, cnt, wv * 64 + lane, r);
    };
    const int nq = S * NW;
#pragma unroll 1
    for (int rr = 0; rr < R; ++rr) {
      const long long j = j0 + rr;
      A cs[C];
#pragma unroll
      for (int c = 0; c < C; ++c) cs[c] = (A)0;
#pragma unroll 1
      for (int q0 = 0; q0 < nq; q0 += 64) {
        const int q = q0 + lane;
        const bool act = q < nq;
        const int ss = q / NW, wv = q - ss * NW;
        const long long gi = rec_index(ss < s ? j : j - 1, ss, wv);
        unsigned long long rv[C][NG];
#pragma unroll
        for (int c = 0; c < C; ++c)
#pragma unroll
          for (int h = 0; h < NG; ++h) rv[c][h] = act ? gran_load(gran + (gi * C + c) * NG + h) : kGranTag;
        bool miss = false;
#pragma unroll
        for (int c = 0; c < C; ++c)
#pragma unroll
          for (int h = 0; h < NG; ++h) miss |= (rv[c][h] >> 32) != 1ull;
#pragma unroll 1
        for (int it = 0; __any(miss) && it < p.spin; ++it) {
          __builtin_amdgcn_s_sleep(2);
          if (miss) {
#pragma unroll
            for (int c = 0; c < C; ++c)
#pragma unroll
              for (int h = 0; h < NG; ++h) rv[c][h] = gran_load(gran + (gi * C + c) * NG + h);
          }
          miss = false;
#pragma unroll
          for (int c = 0; c < C; ++c)
#pragma unroll
            for (int h = 0; h < NG; ++h) miss |= (rv[c][h] >> 32) != 1ull;
        }
        // still untagged: recomputed from the input with the producer's lane
        // mapping and order of operations (the same bits)
        unsigned long long mask = __ballot(miss);
#pragma unroll 1
        while (mask != 0ull) {
          const int l = __builtin_ctzll(mask);
          mask &= mask - 1ull;
          const int qs = __shfl(q, l, 64);
          const int rs = qs / NW;
          SA r[C];
          recompute(rs < s ? j : j - 1, rs, qs - rs * NW, r);
          if (lane == l)
#pragma unroll
            for (int c = 0; c < C; ++c)
#pragma unroll
              for (int h = 0; h < NG; ++h) rv[c][h] = kGranTag | gran_word(r[c], h);
        }
        if (act)
#pragma unroll
          for (int c = 0; c < C; ++c) {
            uint32_t wd[NG];
#pragma unroll
            for (int h = 0; h < NG; ++h) wd[h] = (uint32_t)rv[c][h];
            cs[c] += (A)gran_value<SA>(wd);
          }
      }
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const A cw = readlane(wave_incl_scan(cs[c]), 63);
        if (lane == 0) cbuf[rr & 1][c] = cw;
      }
      __syncthreads();  // the scan's barrier of row rr
    }
    return;
  }

  // ---- the scan waves ----
  auto load_tile = [&](long long j, U_t (&v)[U]) { load_tile_units(j, c0, wcnt, tid, v); };
  auto publish = [&](long long j, const U_t (&v)[U]) {
    SA r[C];
    share_sum(v, wcnt, tid, r);
    publish_record<SA, C>(gran, rec_index(j, s, w), r, lane);
  };
  // one row: P = row j-1, X = row j, N = row j+1, N2 = row j+2 (loaded a step
  // ago, published now: two rows before its siblings' carries need it), N3 <- row j+3
  auto step = [&](int rr, U_t (&P)[U], U_t (&X)[U], U_t (&N2)[U], U_t (&N3)[U]) {
    const long long j = j0 + rr;
    if (rr + 3 < R) load_tile(j + 3, N3);
    if (rr + 2 < R) publish(j + 2, N2);
    SA* tb = tot[rr & 1];
    SA lx[U][C];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      SA run[C];
#pragma unroll
      for (int c = 0; c < C; ++c) run[c] = (SA)0;
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) run[c] += to_acc<SA>(X[u].e[fr * C + c]) - to_acc<SA>(P[u].e[fr * C + c]);
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const SA incl = wave_incl_scan(run[c]);
        lx[u][c] = incl - run[c];
        if (lane == 63) tb[(u * NW + w) * C + c] = incl;
      }
    }
    __syncthreads();
    SA ex[C];
    A cw[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const SA tv = lane < NSEG ? tb[lane * C + c] : (SA)0;
      ex[c] = wave_incl_scan(tv) - tv;
      cw[c] = cbuf[rr & 1][c];
    }
    const long long f0 = j * k + (long long)c0 * F;
    const bool fast = f0 + (long long)wcnt * F <= nframes;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = u * WG + tid;
      A b[C];
#pragma unroll
      for (int c = 0; c < C; ++c) b[c] = cw[c] + (A)(readlane(ex[c], u * NW + wq) + lx[u][c]);
      U_t y;
      SA run[C];
#pragma unroll
      for (int c = 0; c < C; ++c) run[c] = (SA)0;
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) {
          run[c] += to_acc<SA>(X[u].e[fr * C + c]) - to_acc<SA>(P[u].e[fr * C + c]);
          y.e[fr * C + c] = to_out<T, A, DV>(b[c] + (A)run[c], p.o);
        }
      const long long f = f0 + (long long)idx * F;
      if (fast) {
        if (idx < wcnt) IO::template store<(NT & kNtStore) != 0>(out + f * C, y);
      } else if (idx < wcnt) {
#pragma unroll
        for (int fr = 0; fr < F; ++fr)
          if (f + fr < nframes)
#pragma unroll
            for (int c = 0; c < C; ++c) out[(f + fr) * C + c] = y.e[fr * C + c];
      }
    }
  };

  U_t B0[U], B1[U], B2[U], B3[U], B4[U];
  load_tile(j0 - 1, B0);
  load_tile(j0, B1);
  if (R > 1) load_tile(j0 + 1, B2);
  if (R > 2) load_tile(j0 + 2, B3);
  publish(j0 - 1, B0);
  publish(j0, B1);
  if (R > 1) publish(j0 + 1, B2);
#pragma unroll 1
  for (int rr = 0; rr < R; rr += 5) {
    step(rr, B0, B1, B3, B4);
    if (rr + 1 < R) step(rr + 1, B1, B2, B4, B0);
    if (rr + 2 < R) step(rr + 2, B2, B3, B0, B1);
    if (rr + 3 < R) step(rr + 3, B3, B4, B1, B2);
    if (rr + 4 < R) step(rr + 4, B4, B0, B2, B3);
  }
}

}  // namespace mavg
