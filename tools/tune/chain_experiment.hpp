// chain_experiment.hpp -- KEPT-OUT EXPERIMENT (round 3), not part of libmavg.
//
// The chained (decoupled) look-back scan for long windows: each tile scans
// d = x - x[n-k] with its shifted tile staged in LDS, publishes its aggregate
// D(t), and a dedicated fifth "chain" wave folds the nearest published
// inclusive prefix with the aggregates above it (a strict left fold, so fp64
// results are bitwise schedule-independent), then publishes L(t).  Correct:
// every long-window parity test, the forced-schedule bitwise test and the
// dist-2 rounding data passed on MI355X (profiles/r03_tuning/chain/).  Slow:
// 0.25 of HBM peak against 0.68 for the look-ahead scan at 2^30 fp32,
// k=44100.  The phase trace (MAVG_CHAIN_TRACE, chain_trace.py) shows why: the
// look-back is one L2 round trip on data published by tiles running at the
// same moment, 3.5-5.5 us under streaming load, added to every tile's
// ~5-7 us of load + scan; tile lifetime doubles (9-12 us) and with ~5
// workgroups per CU the bytes in flight halve.  The look-ahead scan issues its
// record loads at the start of the tile, on records published D slots
// earlier, so its carry costs no latency.  DESIGN.md "Tried this round".
//
// To rebuild it, include this file after mavg_launch.hpp in a tuning
// translation unit and call dispatch_long<T, A, C, F>(...).
#pragma once

#include "../../digital_signal_processsing_amd/csrc/mavg_launch.hpp"

namespace mavg {

// ----------------------------------------------------------------------------
// The window sum is the inclusive scan of d[n] = x[n] - x[n-k]:
//     W[n] = W[n-1] + d[n],   W[-1] = sum of the history (0 without one).
// So the carry into tile t is the exclusive prefix of the tile aggregates
// D(j) = sum of d over tile j, and a single-pass decoupled look-back scan
// (Merrill & Garland) carries it between workgroups with O(1) work per tile
// whatever k is: each tile stages its own x and its shifted tile x[n-k] (one
// extra read, from L2: that tile was read k/T tiles earlier on this XCD),
// scans d in-tile, publishes its aggregate D(t), looks back for the nearest
// predecessor whose inclusive prefix W(j) is published, and publishes W(t).
// No tile reads k/T records, no tile is read ahead of its workgroup.
//
// Runs.  Tiles run XCD-contiguously (remap mode 1: XCD run x = tiles
// [rs_x, rs_{x+1})), so the shifted tiles are L2 hits; each run is its own
// chain, seeded at its first tile with the window sum in front of it
// (seed_sum: whole-tile records published by the run's first blocks -- "head
// duty" -- plus the partial tile from the stage).  Runs never wait for each
// other.
//
// Determinism.  The chain value is DEFINED as the strict left fold
//     L(rs) = seed + D(rs),   L(j) = L(j-1) + D(j)
// in the accumulator type, and every path computes exactly that fold: a tile
// that finds a published inclusive L(p) adds D(p+1), ..., D(t-1) to it in
// increasing j (never in look-back order), and a published L(p) is itself
// such a fold.  Recomputed aggregates (bounded spin, then the wave redoes
// tile j's scan from global memory with the same lane mapping and order of
// operations) have the same bits.  So fp32 outputs are bitwise the same
// whatever the schedule, and int16 outputs are exact.
//
// Progress never depends on scheduling: a missing aggregate is recomputed
// after `spin` polls; a tile that finds no inclusive at all within `reach`
// predecessors recomputes the run's first link itself (seed + D(rs), the same
// bits tile rs publishes) and folds from there.  All granules are zeroed on
// the stream before every launch (Guideline 16, "Re-initialise every call").
// ----------------------------------------------------------------------------
struct ChainParams {
  const void* in;
  void* out;
  const void* hist;
  long long nframes;
  int k;
  int halo_units;   // ceil(k / F): the shifted stage starts halo_units*F frames before the tile
  int xk_off;       // (-k*C) mod VE
  int hrec;         // record slots per run: whole tiles a seed window can hold, ceil(k/T) + 1
  int spin;         // polls of an unpublished granule before recomputing it
  int reach;        // predecessors searched for a published inclusive before recomputing the run's first link
  int pre;          // frames in front of `in` that are readable signal (load_elem)
  int eio;          // frame-unit launch on element-aligned pointers (UnitIO::gload)
  unsigned long long* agg;  // [ntiles][C][NGA] tile aggregates D(t)
  unsigned long long* inc;  // [ntiles][C][NGA] inclusive prefixes L(t)
  unsigned long long* rec;  // [8][hrec][NW][C][NGS] seed records: per-wave shares of whole-tile sums
  unsigned* front;          // [8] per run: 1 + the highest run position whose inclusive is published
  void* stats;              // MAVG_AHEAD_STATS builds only: {recomputes, polls that waited}
  unsigned long long* trace;  // MAVG_CHAIN_TRACE builds only: [ntiles][8] timestamps (chain_trace.py)
  OutParams o;
};


// Load tile j's link (all channels) into this lane: true when every granule
// is published.
template <typename V, int C>
__device__ __forceinline__ bool link_load(const gran_t* arr, long long j, V (&v)[C]) {
  constexpr int NG = GranCount<V>::n;
  bool ok = true;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    uint32_t wd[NG];
#pragma unroll
    for (int h = 0; h < NG; ++h) {
      const unsigned long long g = gran_load(arr + (j * C + c) * NG + h);
      ok &= (g >> 32) == 1ull;
      wd[h] = (uint32_t)g;
    }
    v[c] = gran_value<V>(wd);
  }
  return ok;
}
// lanes 0 .. C*NG-1 each store one granule of slot j (the same form as publish_record)
template <typename V, int C>
__device__ __forceinline__ void link_store(gran_t* arr, long long j, const V (&v)[C], int lane) {
  publish_record<V, C>(arr, j, v, lane);
}

// MAVG_CHAIN_TRACE (tuning builds only, tools/tune/chain_trace.py): per tile,
// 100-MHz wall-clock stamps of the phases and the look-back's outcome
#ifdef MAVG_CHAIN_TRACE
#define MAVG_TRACE(slot, v) (p.trace[(unsigned long long)tile * 8 + (slot)] = (unsigned long long)(v))
#define MAVG_NOW() __builtin_amdgcn_s_memrealtime()
#else
#define MAVG_TRACE(slot, v) ((void)0)
#define MAVG_NOW() 0ull
#endif

// A workgroup barrier for LDS hand-offs only: LDS writes drained
// (lgkmcnt(0)), then s_barrier.  __syncthreads() also drains every global
// store and atomic (its release fence waits on vmcnt), which would put the
// chain wave's link stores on the tile waves' critical path.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xc07f);  // gfx9 encoding: lgkmcnt(0), vmcnt/expcnt untouched
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// s_sleep takes an immediate: n units of 64 cycles
__device__ __forceinline__ void sleep_units(int n) {
  for (; n > 0; --n) __builtin_amdgcn_s_sleep(1);
}
__device__ __forceinline__ unsigned frontier_load(unsigned* f) {
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// L(t-1) from the nearest inclusive L(t-1-ls) (`top`) and the aggregates of
// lanes ls-1 .. 0 (tiles t-ls .. t-1).  fp64: the strict left fold in
// increasing tile order, the chain's definition; integers: exact in any order,
// one wave reduction.
__device__ __forceinline__ double fold_window(double top, double av, int ls, int lane) {
  double acc = top;
#pragma unroll 1
  for (int l = ls - 1; l >= 0; --l) acc += readlane(av, l);
  return acc;
}
template <typename I>
__device__ __forceinline__ I fold_window(I top, I av, int ls, int lane) {
  return top + readlane(wave_incl_scan(lane < ls ? av : (I)0), 63);
}

__device__ __forceinline__ double readlane_v(double v, int l) { return readlane(v, l); }
__device__ __forceinline__ int32_t readlane_v(int32_t v, int l) { return readlane(v, l); }
__device__ __forceinline__ int64_t readlane_v(int64_t v, int l) { return readlane(v, l); }

// One unit's in-lane total of d = x - x[n-k], in the kernel's order of
// operations (RC: run += x - xk from 0; otherwise the running prefix v).
template <typename T, typename SA, int C, int F, bool RC>
__device__ __forceinline__ void unit_total(const Unit<T, F * C>& xu, const Unit<T, F * C>& xk, SA (&run)[C]) {
  if constexpr (RC) {
#pragma unroll
    for (int c = 0; c < C; ++c) run[c] = (SA)0;
#pragma unroll
    for (int fr = 0; fr < F; ++fr)
#pragma unroll
      for (int c = 0; c < C; ++c) run[c] += to_acc<SA>(xu.e[fr * C + c]) - to_acc<SA>(xk.e[fr * C + c]);
  } else {
#pragma unroll
    for (int fr = 0; fr < F; ++fr)
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const SA d = to_acc<SA>(xu.e[fr * C + c]) - to_acc<SA>(xk.e[fr * C + c]);
        run[c] = fr == 0 ? d : run[c] + d;
      }
  }
}

// Per-wave share of a whole tile's x sum (a seed record): lane l sums units
// u*WG + wv*64 + l over u, frames and channels, then one DPP wave scan.  Tiles
// before frame 0 (history) or past the end load element by element.
// LEAN: one unit in registers at a time (the rare recompute path: fewer
// registers, same additions in the same order, so the same bits).
template <typename T, typename SA, int C, int F, int U, bool LEAN = false>
__device__ __forceinline__ void record_share(const T* __restrict__ in, const T* __restrict__ hist, long long q, int wv,
                                             int lane, const ChainParams& p, SA (&r)[C]) {
  constexpr int VE = F * C;
  constexpr int TF = kWG * F * U;
  constexpr int UB = LEAN ? 1 : U;  // units in flight
  using IO = UnitIO<T, VE>;
  const bool fast = q >= 0 && (q + 1) * TF <= p.nframes;
  const bool eio = F == 1 && p.eio != 0;
  SA ls[C];
#pragma unroll
  for (int c = 0; c < C; ++c) ls[c] = (SA)0;
#pragma unroll 1
  for (int u0 = 0; u0 < U; u0 += UB) {
    Unit<T, VE> xs[UB];
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      const long long f = q * TF + (long long)((u0 + b) * kWG + wv * 64 + lane) * F;
      if (fast) {
        xs[b] = IO::gload(in + f * C, eio);
      } else {
#pragma unroll
        for (int fr = 0; fr < F; ++fr)
#pragma unroll
          for (int c = 0; c < C; ++c) xs[b].e[fr * C + c] = load_elem(in, hist, f + fr, c, C, p.nframes, p.k, p.pre);
      }
    }
#pragma unroll
    for (int b = 0; b < UB; ++b)
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) ls[c] += to_acc<SA>(xs[b].e[fr * C + c]);
  }
#pragma unroll
  for (int c = 0; c < C; ++c) r[c] = readlane(wave_incl_scan(ls[c]), 63);
}

// Recompute tile j's aggregate D(j) with one wave, bitwise as tile j computes
// it: the same units, the same in-lane order (unit_total), the same wave
// scans, the segment totals scanned across lanes in segment order.
template <typename T, typename A, int C, int F, int U, bool RC>
__device__ __forceinline__ void recompute_aggregate(const T* __restrict__ in, const T* __restrict__ hist, long long j,
                                                 int lane, const ChainParams& p,
                                                 typename ScanAcc<T, A>::type (&dj)[C]) {
  using SA = typename ScanAcc<T, A>::type;
  constexpr int NW = kWG / 64;
  constexpr int VE = F * C;
  constexpr int TF = kWG * F * U;
  constexpr int NSEG = U * NW;
  using IO = UnitIO<T, VE>;
  const int k = p.k;
  const bool eio = F == 1 && p.eio != 0;
  const bool xfast = (j + 1) * TF <= p.nframes;
  SA seg[C];
#pragma unroll
  for (int c = 0; c < C; ++c) seg[c] = (SA)0;
#pragma unroll 1
  for (int s = 0; s < NSEG; ++s) {
    const int u = s / NW, wv = s % NW;
    const long long f = j * TF + (long long)(u * kWG + wv * 64 + lane) * F;
    Unit<T, VE> xu, xk;
    if (xfast) {
      xu = IO::gload(in + f * C, eio);
    } else {
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) xu.e[fr * C + c] = load_elem(in, hist, f + fr, c, C, p.nframes, k, p.pre);
    }
#pragma unroll
    for (int fr = 0; fr < F; ++fr)
#pragma unroll
      for (int c = 0; c < C; ++c) xk.e[fr * C + c] = load_elem(in, hist, f + fr - k, c, C, p.nframes, k, p.pre);
    SA run[C];
    unit_total<T, SA, C, F, RC>(xu, xk, run);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const SA segtot = readlane(wave_incl_scan(run[c]), 63);
      if (lane == s) seg[c] = segtot;
    }
  }
#pragma unroll
  for (int c = 0; c < C; ++c) dj[c] = readlane(wave_incl_scan(seg[c]), NSEG - 1);
}

// The window sum in front of run start rs (one wave, fixed order): the
// partial tile [a, jlo*T) -- from the caller's LDS stage (`stage`, first
// frame h0) or from global memory (stage == nullptr) -- and the per-wave
// records of the whole tiles [jlo, rs), lane l taking partial frames a+l,
// a+l+64, ... then records l, l+64, ..., one wave scan at the end.
template <typename T, typename A, int C, int F, int U>
__device__ __forceinline__ void seed_sum(const T* __restrict__ in, const T* __restrict__ hist, long long rs, int run,
                                      const T* stage, long long h0, int lane, const ChainParams& p, A (&seed)[C]) {
  using SA = typename ScanAcc<T, A>::type;
  constexpr int NW = kWG / 64;
  constexpr int TF = kWG * F * U;
  constexpr int NGS = GranCount<SA>::n;
  const int k = p.k;
  const bool has_hist = p.hist != nullptr || p.pre > 0;
  const long long a = rs * TF - k;
  long long jlo;
  if (a >= 0) jlo = (a + TF - 1) / TF;
  else jlo = has_hist ? -((-a) / TF) : 0;  // ceil(a / T) for a < 0
  const long long plo = (a >= 0 || has_hist) ? a : 0;  // partial frames [plo, jlo*T)
  A acc[C];
#pragma unroll
  for (int c = 0; c < C; ++c) acc[c] = (A)0;
#pragma unroll 4
  for (long long f = plo + lane; f < jlo * TF; f += 64)
#pragma unroll
    for (int c = 0; c < C; ++c)
      acc[c] += to_acc<A>(stage != nullptr ? stage[(f - h0) * C + c]
                                           : load_elem(in, hist, f, c, C, p.nframes, k, p.pre));
  // records: slot (q - jlo) * NW + wave share, published by the run's head duty
  const int nrec = (int)(rs - jlo) * NW;
  gran_t* rec = (gran_t*)p.rec + (long long)run * p.hrec * NW * C * NGS;
#pragma unroll 1
  for (int r0 = 0; r0 < nrec; r0 += 64) {
    const int r = r0 + lane;
    const bool act = r < nrec;
    SA v[C];
    bool ok = act ? link_load<SA, C>(rec, r, v) : true;
#pragma unroll 1
    for (int it = 0; !__all(ok) && it < p.spin; ++it) {
      __builtin_amdgcn_s_sleep(2);
      if (!ok) ok = link_load<SA, C>(rec, r, v);
    }
    unsigned long long miss = __ballot(!ok);
#pragma unroll 1
    while (miss != 0ull) {  // the head-duty block has not published: recompute the share
      const int l = __builtin_ctzll(miss);
      miss &= miss - 1ull;
      const int rl = r0 + l;
      SA sh[C];
      record_share<T, SA, C, F, U, true>(in, hist, jlo + rl / NW, rl % NW, lane, p, sh);
      if (lane == l)
#pragma unroll
        for (int c = 0; c < C; ++c) v[c] = sh[c];
#ifdef MAVG_AHEAD_STATS
      if (lane == 0) atomicAdd(reinterpret_cast<unsigned int*>(p.stats), 1u);
#endif
    }
    if (act)
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] += (A)v[c];
  }
#pragma unroll
  for (int c = 0; c < C; ++c) seed[c] = readlane(wave_incl_scan(acc[c]), 63);
}

// L(t-1) the long way, for a tile that found no published inclusive within
// its 64 nearest predecessors: the run's seed, then D(rs), ..., D(t-1) in
// order, each the published aggregate or recomputed (the strict left fold
// that defines the chain, so the same bits as any other path).
template <typename T, typename A, int C, int F, int U, bool RC>
__device__ __forceinline__ void chain_from_seed(const T* __restrict__ in, const T* __restrict__ hist, long long rs,
                                             int run, long long tile, int lane, const ChainParams& p, A (&acc)[C]) {
  using SA = typename ScanAcc<T, A>::type;
  const gran_t* agg = (const gran_t*)p.agg;
  seed_sum<T, A, C, F, U>(in, hist, rs, run, nullptr, 0, lane, p, acc);
#pragma unroll 1
  for (long long jb = rs; jb < tile; jb += 64) {
    const long long j = jb + lane;
    A av[C];
    const bool ok = j < tile && link_load<A, C>(agg, j, av);
    unsigned long long miss = __ballot(j < tile && !ok);
#pragma unroll 1
    while (miss != 0ull) {
      const int l = __builtin_ctzll(miss);
      miss &= miss - 1ull;
      SA dj[C];
      recompute_aggregate<T, A, C, F, U, RC>(in, hist, jb + l, lane, p, dj);
      if (lane == l)
#pragma unroll
        for (int c = 0; c < C; ++c) av[c] = (A)dj[c];
    }
    const int n = (int)min((long long)64, tile - jb);
#pragma unroll 1
    for (int l = 0; l < n; ++l)
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] += readlane_v(av[c], l);
  }
}

// The chain wave: after the tile waves' segment totals are in LDS, D(t), the
// look-back, L(t) and the carry for the tile waves.  A wave of its own, so the
// look-back's registers never coexist with a tile wave's tile registers (the
// kernel's VGPR count is the larger of the two paths, not their sum).
template <typename T, typename A, int C, int F, int U, bool RC>
__device__ __forceinline__ void chain_wave(const ChainParams& p, const T* __restrict__ in, const T* __restrict__ hist,
                                           const T* stage, const typename ScanAcc<T, A>::type* tot, A* basep,
                                           long long tile, long long rs, int run, long long h0, int lane) {
  using SA = typename ScanAcc<T, A>::type;
  constexpr int NW = kWG / 64;
  constexpr int NSEG = U * NW;
  gran_t* agg = (gran_t*)p.agg;
  gran_t* inc = (gran_t*)p.inc;
  // the tile aggregate D(t): the segment totals scanned across lanes in
  // segment order (the same scan the tile waves use for their prefixes)
  SA dt[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const SA tv = lane < NSEG ? tot[lane * C + c] : (SA)0;
    dt[c] = readlane(wave_incl_scan(tv), NSEG - 1);
  }
  const long long i = tile - rs;  // position in the run's chain
  if (lane == 0) MAVG_TRACE(2, MAVG_NOW());
  A base[C];
  if (i == 0) {
    seed_sum<T, A, C, F, U>(in, hist, rs, run, stage, h0, lane, p, base);
  } else {
    {
      A dA[C];
#pragma unroll
      for (int c = 0; c < C; ++c) dA[c] = (A)dt[c];
      link_store<A, C>(agg, tile, dA, lane);
    }
    // The 64 nearest predecessors' inclusive and aggregate links in one
    // round of loads: the nearest published inclusive L(t-1-ls), and every
    // aggregate above it, fold in registers.  No inclusive in the window
    // (the run's frontier is further back): poll the run's frontier word
    // -- one load per poll, with backoff, never the whole window (a storm of
    // window re-reads saturates the XCD's L2) -- until it comes within 64
    // tiles, then reload the window.  After `spin` rounds without one,
    // recompute the chain from the run's seed (the same fold, so the same
    // bits).
    const long long j = tile - 1 - lane;
    const bool act = j >= rs && lane < p.reach;
    const long long jc = act ? j : tile - 1;  // every lane loads (one round for both arrays), inactive ones a valid slot
    const unsigned need = (unsigned)max(1LL, i + 1 - 64);  // frontier value that puts an inclusive in the window
#pragma unroll 1
    for (int it = 0;;) {
      A iv[C], av[C];
      const bool hl = link_load<A, C>(inc, jc, iv);
      const bool al = link_load<A, C>(agg, jc, av);
      const bool hi = act && hl;
      bool ha = act && al;
      const unsigned long long mi = __ballot(hi);
      if (mi != 0ull) {
        const int ls = __builtin_ctzll(mi);
        const unsigned long long below = ls == 0 ? 0ull : ((1ull << ls) - 1ull);
#pragma unroll 1
        for (int sp = 0, b = 1; (__ballot(ha) & below) != below && sp < p.spin; ++sp, b = min(2 * b, 32)) {
#ifdef MAVG_AHEAD_STATS
          if (lane == 0) atomicAdd(reinterpret_cast<unsigned int*>(p.stats) + 1, 1u);
#endif
          sleep_units(b);
          if (!ha && lane < ls) ha = link_load<A, C>(agg, j, av);
        }
        unsigned long long miss = below & ~__ballot(ha);
#pragma unroll 1
        while (miss != 0ull) {
          const int l = __builtin_ctzll(miss);
          miss &= miss - 1ull;
          SA dj[C];
          recompute_aggregate<T, A, C, F, U, RC>(in, hist, tile - 1 - l, lane, p, dj);
          if (lane == l)
#pragma unroll
            for (int c = 0; c < C; ++c) av[c] = (A)dj[c];
#ifdef MAVG_AHEAD_STATS
          if (lane == 0) atomicAdd(reinterpret_cast<unsigned int*>(p.stats), 1u);
#endif
        }
#pragma unroll
        for (int c = 0; c < C; ++c) base[c] = fold_window(readlane_v(iv[c], ls), av[c], ls, lane);
        if (lane == 0) MAVG_TRACE(6, (unsigned long long)ls | ((unsigned long long)it << 32));
        break;
      }
      if (p.reach == 0 || it >= p.spin) {
        chain_from_seed<T, A, C, F, U, RC>(in, hist, rs, run, tile, lane, p, base);
#ifdef MAVG_AHEAD_STATS
        if (lane == 0) atomicAdd(reinterpret_cast<unsigned int*>(p.stats), 1u);
#endif
        break;
      }
#pragma unroll 1
      for (int b = 1; it < p.spin; b = min(2 * b, 64)) {
        ++it;
        sleep_units(b);
        if (frontier_load(p.front + run) >= need) break;
      }
    }
  }
  A lt[C];
#pragma unroll
  for (int c = 0; c < C; ++c) lt[c] = base[c] + (A)dt[c];
  link_store<A, C>(inc, tile, lt, lane);
  // advance the run's frontier (monotonic): waiting tiles poll this one word
  if (lane == 0) {
    MAVG_TRACE(3, MAVG_NOW());
    __hip_atomic_fetch_max(p.front + run, (unsigned)(tile - rs + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int c = 0; c < C; ++c) basep[c] = base[c];
  }
}

// NT: kNtLoad (tile loads), kNtHalo (shifted-tile loads), kNtStore (outputs).
// RC: keep the tile's registers across the barriers and rebuild the in-lane
//     prefix at the output (fewer live fp64 accumulators).
// DMA: stage interior shifted tiles by LDS-DMA (16-B units).
// DV: the int16 output division (to_out).
template <typename T, typename A, int C, int F, int U, int NT, bool RC = false, bool DMA = true, int DV = 0>
__global__ __launch_bounds__(kWG + 64) void chain_scan_kernel(ChainParams p) {
  constexpr int WG = kWG;  // tile waves; wave NW (threads WG .. WG+63) is the chain wave
  constexpr int NW = WG / 64;
  constexpr int VE = F * C;
  constexpr int TF = WG * F * U;
  constexpr int NSEG = U * NW;
  constexpr int kStageUnits = U * WG + 1;
  constexpr int kStageBytes = ((kStageUnits * VE * (int)sizeof(T)) + 15) & ~15;
  using IO = UnitIO<T, VE>;
  using U_t = Unit<T, VE>;
  using SA = typename ScanAcc<T, A>::type;
  constexpr int NGS = GranCount<SA>::n;
  constexpr bool kDma = DMA && IO::kVec && VE * (int)sizeof(T) == 16;

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* stage = reinterpret_cast<T*>(smem);
  SA* tot = reinterpret_cast<SA*>(smem + kStageBytes);  // [NSEG][C] segment totals
  A* basep = reinterpret_cast<A*>(tot + NSEG * C);      // [C] the carry L(t-1), from the chain wave

  const T* __restrict__ in = static_cast<const T*>(p.in);
  T* __restrict__ out = static_cast<T*>(p.out);
  const T* __restrict__ hist = static_cast<const T*>(p.hist);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int wq = __builtin_amdgcn_readfirstlane(w);
  const int k = p.k;
  const long long nframes = p.nframes;
  const int pre = p.pre;
  const bool eio = F == 1 && p.eio != 0;

  const unsigned nb = gridDim.x;
  const long long tile = remap_tile(blockIdx.x, nb, 1);
  const int run = (int)(blockIdx.x & 7u);
  const unsigned slot = blockIdx.x >> 3;
  const long long rs = run_start((unsigned)run, nb);  // first tile of this XCD run (= tile - slot)
  const long long t0 = tile * TF;
  const int Ha = p.halo_units * F;
  const long long h0 = t0 - Ha;
  const bool tile_full = (t0 + TF <= nframes);
  MAVG_DCHECK(tile >= 0 && tile < (long long)nb && tile == rs + slot, "chain tile index", tile, slot);

  if (wq == NW) {  // the chain wave: no tile registers
    __syncthreads();  // A: the shifted stage is complete
    lds_barrier();    // B: the segment totals are in LDS
    chain_wave<T, A, C, F, U, RC>(p, in, hist, stage, tot, basep, tile, rs, run, h0, lane);
    lds_barrier();    // C: the carry is in LDS (the link stores drain on their own)
    return;
  }

  if (tid == 0) MAVG_TRACE(0, MAVG_NOW());
  // ---- 1. loads: the tile to registers, the shifted tile to the LDS stage ----
  U_t x[U];
  if (tile_full) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      x[u] = IO::template gload<(NT & kNtLoad) != 0>(in + (t0 + (long long)(u * WG + tid) * F) * C, eio);
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long f = t0 + (long long)(u * WG + tid) * F;
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) x[u].e[fr * C + c] = load_elem(in, hist, f + fr, c, C, nframes, k, pre);
    }
  }
  const bool stage_fast = !eio && h0 >= 0 && h0 + (long long)kStageUnits * F <= nframes;
  if (kDma && stage_fast) {
    if constexpr (kDma) {
      unsigned char* sb = reinterpret_cast<unsigned char*>(stage);
#pragma unroll
      for (int u = 0; u < U; ++u)
        glds16<(NT & kNtHalo) != 0>(in + (h0 + (long long)(u * WG + tid) * F) * C, sb + (u * WG + wq * 64) * 16);
      if (tid == 0) glds16<(NT & kNtHalo) != 0>(in + (h0 + (long long)(U * WG) * F) * C, sb + (U * WG) * 16);
    }
  } else if (stage_fast) {
    stage_shifted_tile<T, C, F, U, WG, NT>(in, hist, stage, h0, nframes, k, pre, eio, tid);
  } else {
#pragma unroll 1
    for (int j = tid; j < kStageUnits; j += WG) {
      const long long f = h0 + (long long)j * F;
      U_t h;
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) h.e[fr * C + c] = load_elem(in, hist, f + fr, c, C, nframes, k, pre);
      IO::store(stage + j * VE, h);
    }
  }

  // ---- head duty: the first blocks of run x publish the per-wave shares of
  //      the whole tiles in the seed window of run x (seed_sum) ----
  {
    const bool has_hist = p.hist != nullptr || pre > 0;
    const long long a = rs * TF - k;
    const long long jlo = a >= 0 ? (a + TF - 1) / TF : (has_hist ? -((-a) / TF) : 0);
    if ((long long)slot < rs - jlo) {
      const long long q = jlo + slot;
      SA r[C];
      record_share<T, SA, C, F, U>(in, hist, q, w, lane, p, r);
      gran_t* rec = (gran_t*)p.rec + (long long)run * p.hrec * NW * C * NGS;
      MAVG_DCHECK(slot * NW + w < (unsigned)(p.hrec * NW), "seed record slot", slot, p.hrec);
      publish_record<SA, C>(rec, (long long)slot * NW + w, r, lane);
    }
  }
  __syncthreads();

  if (tid == 0) MAVG_TRACE(1, MAVG_NOW());
  // ---- 2. d = x - x[n-k]; in-lane, wave and segment scans ----
  auto stage_xk = [&](int j) -> U_t {
    const int e = (Ha + j * F - k) * C;  // stage element of x[n-k]
    U_t xk;
    if constexpr (IO::kVec) {
      if (p.xk_off == 0) {
        MAVG_DCHECK(e >= 0 && e + VE <= kStageUnits * VE, "chain x[n-k] stage index", e, j);
        xk = IO::load(stage + e);
      } else {
        const int e_lo = e - p.xk_off;
        MAVG_DCHECK(e_lo >= 0 && e_lo + 2 * VE <= kStageUnits * VE, "chain x[n-k] extraction", e_lo, j);
        U_t a0 = IO::load_whole(stage + e_lo);
        U_t a1 = IO::load_whole(stage + e_lo + VE);
        xk = extract(a0, a1, p.xk_off);
      }
    } else {
#pragma unroll
      for (int i = 0; i < VE; ++i) xk.e[i] = stage[e + i];
    }
    return xk;
  };
  SA v[RC ? 1 : U][F][C];
  SA lx[U][C];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const U_t xk = stage_xk(u * WG + tid);
    SA run_[C];
    if constexpr (RC) {
      unit_total<T, SA, C, F, true>(x[u], xk, run_);
    } else {
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) {
          const SA d = to_acc<SA>(x[u].e[fr * C + c]) - to_acc<SA>(xk.e[fr * C + c]);
          v[u][fr][c] = fr == 0 ? d : v[u][fr - 1][c] + d;
        }
#pragma unroll
      for (int c = 0; c < C; ++c) run_[c] = v[u][F - 1][c];
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const SA incl = wave_incl_scan(run_[c]);
      lx[u][c] = incl - run_[c];
      const SA segtot = readlane(incl, 63);
      if (lane == 0) tot[(u * NW + w) * C + c] = segtot;
    }
  }
  lds_barrier();  // B: segment totals in LDS

  // ---- 3. segment prefixes (the tile waves) ----
  static_assert(NSEG <= 64, "segment totals are scanned across one wave");
  SA ex[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const SA tv = lane < NSEG ? tot[lane * C + c] : (SA)0;
    ex[c] = wave_incl_scan(tv) - tv;
  }
  lds_barrier();  // C: the chain wave has written the carry
  if (tid == 0) MAVG_TRACE(4, MAVG_NOW());

  // ---- 4. carry + earlier segments; outputs ----
  A w0[C];
#pragma unroll
  for (int c = 0; c < C; ++c) w0[c] = basep[c];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long f = t0 + (long long)(u * WG + tid) * F;
    A b[C];
#pragma unroll
    for (int c = 0; c < C; ++c) b[c] = w0[c] + (A)(readlane(ex[c], u * NW + wq) + lx[u][c]);
    U_t y;
    if constexpr (RC) {
      const U_t xk = stage_xk(u * WG + tid);
      SA run_[C];
#pragma unroll
      for (int c = 0; c < C; ++c) run_[c] = (SA)0;
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) {
          run_[c] += to_acc<SA>(x[u].e[fr * C + c]) - to_acc<SA>(xk.e[fr * C + c]);
          y.e[fr * C + c] = to_out<T, A, DV>(b[c] + (A)run_[c], p.o);
        }
    } else {
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) y.e[fr * C + c] = to_out<T, A, DV>(b[c] + (A)v[u][fr][c], p.o);
    }
    if (tile_full) {
      IO::template gstore<(NT & kNtStore) != 0>(out + f * C, y, eio);
    } else {
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
        if (f + fr < nframes)
#pragma unroll
          for (int c = 0; c < C; ++c) out[(f + fr) * C + c] = y.e[fr * C + c];
    }
  }
  if (tid == 0) MAVG_TRACE(5, MAVG_NOW());
}


// chained look-back scan (mavg_chain.hpp): zero the link and record
// granules, then one launch; tile t publishes its aggregate D(t), folds the
// nearest published inclusive prefix with the aggregates above it, and
// publishes L(t).
// Workspace (8-B granules, one block from the start, padded to 16 bytes for
// the memset's fast form): aggregates and inclusive prefixes, one slot per
// (tile, channel, 32-bit word of the accumulator), then the run seeds'
// per-wave records (8 runs x (k/T + 2) tiles x 4 waves), preceded by 64
// bytes of run frontier words and followed by 16 bytes of launch statistics
// (MAVG_AHEAD_STATS builds only).
template <typename T, typename A, int C, int F, int U>
struct ChainLayout {
  using SA = typename ScanAcc<T, A>::type;
  static constexpr int TF = kWG * F * U;
  long long ntiles, hrec;
  size_t link_gran, rec_gran;
  ChainLayout(long long nframes, int k) {
    ntiles = (nframes + TF - 1) / TF;
    hrec = (long long)k / TF + 2;
    link_gran = (size_t)ntiles * C * GranCount<A>::n;
    rec_gran = (size_t)8 * hrec * kNW * C * GranCount<SA>::n;
  }
  // 64 bytes of run frontier words first, then the granules, then 16 bytes of stats
  size_t bytes() const { return 64 + ((2 * link_gran + rec_gran) * 8 + 15) / 16 * 16 + 16 + trace_bytes(); }
#ifdef MAVG_CHAIN_TRACE
  size_t trace_bytes() const { return (size_t)ntiles * 64; }  // tuning builds: 8 stamps per tile, at the end
#else
  size_t trace_bytes() const { return 0; }
#endif
};
template <typename T, typename A, int C, int F, int U, int NT, bool RC, bool DMA, int DV = 0>
int launch_chain_scan(const Sig& sg, int k, hipStream_t st, Workspace ws) {
  const long long nframes = sg.nframes;
  int reach = 1 << 30, spin = kAheadSpin;
  {
    const int t = g_test_ahead_slots.load(std::memory_order_relaxed);
    if (t >= 0) reach = t;
    const int s = g_test_ahead_spin.load(std::memory_order_relaxed);
    if (s >= 0) spin = s;
  }
  constexpr int TF = kWG * F * U;
  constexpr int VE = F * C;
  constexpr int NSEG = U * kNW;
  using SA = typename ScanAcc<T, A>::type;
  constexpr size_t kStageBytes = (((size_t)(U * kWG + 1) * VE * sizeof(T)) + 15) & ~(size_t)15;
  const ChainLayout<T, A, C, F, U> L(nframes, k);
  if (L.ntiles > 0x7fffffffLL) return MAVG_ERR_UNSUPPORTED;
  const size_t need = L.bytes();
  const size_t lds = kStageBytes + (size_t)NSEG * C * sizeof(SA) + (size_t)C * sizeof(A) + 8;
  if (lds > kLdsBudget) return MAVG_ERR_UNSUPPORTED;
  if (g_plan) {
    snprintf(g_plan->text, sizeof(g_plan->text),
             "chain_scan<%s,acc=%s,C=%d,F=%d,U=%d,nt=%d,rc=%d,dma=%d,dv=%d> grid=%lld block=%d lds=%zu "
             "tile_frames=%d remap=1 ws=%zu",
             type_name<T>(), type_name<A>(), C, F, U, NT, (int)RC, (int)DMA, DV, L.ntiles, kWG + 64, lds, TF, need);
    g_plan->ws_bytes = need;
    return MAVG_OK;
  }
  if (ws.ptr == nullptr || ws.bytes < need) return MAVG_ERR_WORKSPACE;
  if ((reinterpret_cast<uintptr_t>(ws.ptr) & 15u) != 0) return MAVG_ERR_MISALIGNED;
  if (hipMemsetAsync(ws.ptr, 0, need, st) != hipSuccess) return MAVG_ERR_HIP;
  unsigned long long* g = reinterpret_cast<unsigned long long*>(static_cast<unsigned char*>(ws.ptr) + 64);
  ChainParams p{};
  p.in = sg.in;
  p.out = sg.out;
  p.hist = sg.hist;
  p.nframes = nframes;
  p.k = k;
  p.halo_units = (k + F - 1) / F;
  p.xk_off = (int)((VE - ((long long)k * C) % VE) % VE);
  p.hrec = (int)L.hrec;
  p.spin = spin;
  p.reach = reach;
  p.pre = sg.pre;
  p.eio = sg.eio;
  p.agg = g;
  p.inc = g + L.link_gran;
  p.rec = g + 2 * L.link_gran;
  p.front = static_cast<unsigned*>(ws.ptr);
  p.stats = static_cast<unsigned char*>(ws.ptr) + need - 16 - L.trace_bytes();
  p.trace = reinterpret_cast<unsigned long long*>(static_cast<unsigned char*>(ws.ptr) + need - L.trace_bytes());
  p.o = make_out_params(k);
  // four tile waves + the chain wave
  hipLaunchKernelGGL((chain_scan_kernel<T, A, C, F, U, NT, RC, DMA, DV>), dim3((unsigned)L.ntiles), dim3(kWG + 64), lds,
                     st, p);
  return hipGetLastError() == hipSuccess ? MAVG_OK : MAVG_ERR_HIP;
}

// The long-window scan: the chained look-back scan with 4096-frame tiles
// (U=4 x 16-B units), LDS-DMA shifted stage, non-temporal shifted-tile loads
// and output stores (its last use), default-policy tile loads (the tile is
// the shifted tile of tile t + k/T, an L2 hit if it stays); fp32 mono keeps
// the tile in registers across the barriers (RC).
template <typename T, typename A, int C, int F>
int dispatch_long(const Sig& sg, int k, hipStream_t st, Workspace ws) {
  constexpr int U = 4;
  constexpr int kNtA = kNtStore | kNtHalo;
  constexpr bool kRC = sizeof(T) == 4 && C == 1;
  return launch_chain_scan<T, A, C, F, U, kNtA, kRC, true>(sg, k, st, ws);
}


}  // namespace mavg
