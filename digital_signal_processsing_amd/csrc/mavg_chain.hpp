// mavg_chain.hpp -- the chained look-back scan (chain_scan_kernel): windows too
// long for an LDS-staged halo.  Replaces the carry of the reference's
// recursive_blelloch (basics/blelloch_scan_averager.cu:134-167) and the
// blelloch_uniform_add pass (:17-36) for any window length.
#pragma once

#include "mavg_lookback.hpp"

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
  void* stats;              // MAVG_AHEAD_STATS builds only: {recomputes, polls that waited}
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

// NT: kNtLoad (tile loads), kNtHalo (shifted-tile loads), kNtStore (outputs).
// RC: keep the tile's registers across the barriers and rebuild the in-lane
//     prefix at the output (fewer live fp64 accumulators).
// DMA: stage interior shifted tiles by LDS-DMA (16-B units).
// DV: the int16 output division (to_out).
template <typename T, typename A, int C, int F, int U, int NT, bool RC = false, bool DMA = true, int DV = 0>
__global__ __launch_bounds__(kWG) __attribute__((amdgpu_waves_per_eu(5))) void chain_scan_kernel(ChainParams p) {
  constexpr int WG = kWG;
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
  A* basep = reinterpret_cast<A*>(tot + NSEG * C);      // [C] the carry L(t-1), from wave 0

  const T* __restrict__ in = static_cast<const T*>(p.in);
  T* __restrict__ out = static_cast<T*>(p.out);
  const T* __restrict__ hist = static_cast<const T*>(p.hist);
  gran_t* agg = (gran_t*)p.agg;
  gran_t* inc = (gran_t*)p.inc;
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
  __syncthreads();

  // ---- 3. segment prefixes (every wave) and the tile aggregate D(t) ----
  static_assert(NSEG <= 64, "segment totals are scanned across one wave");
  SA ex[C], dt[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const SA tv = lane < NSEG ? tot[lane * C + c] : (SA)0;
    const SA incl = wave_incl_scan(tv);
    ex[c] = incl - tv;
    dt[c] = readlane(incl, NSEG - 1);
  }

  // ---- 4. the chain (wave 0): publish D(t), find L(t-1), publish L(t) ----
  if (wq == 0) {
    const long long i = tile - rs;  // position in the run's chain
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
      // aggregate above it, fold in registers.  Until one of them publishes
      // an inclusive, poll (bounded); then recompute the run's chain from its
      // seed (the pathological path: the same fold, so the same bits).
      const long long j = tile - 1 - lane;
      const bool act = j >= rs;
#pragma unroll 1
      for (int it = 0;; ++it) {
        A iv[C], av[C];
        const bool hi = act && link_load<A, C>(inc, j, iv);
        bool ha = act && link_load<A, C>(agg, j, av);
        const unsigned long long mi = __ballot(hi);
        if (mi != 0ull && __builtin_ctzll(mi) < p.reach) {
          const int ls = __builtin_ctzll(mi);
          const unsigned long long below = ls == 0 ? 0ull : ((1ull << ls) - 1ull);
#pragma unroll 1
          for (int sp = 0; (__ballot(ha) & below) != below && sp < p.spin; ++sp) {
#ifdef MAVG_AHEAD_STATS
            if (lane == 0) atomicAdd(reinterpret_cast<unsigned int*>(p.stats) + 1, 1u);
#endif
            __builtin_amdgcn_s_sleep(2);
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
          for (int c = 0; c < C; ++c) {
            A acc = readlane_v(iv[c], ls);
#pragma unroll 1
            for (int l = ls - 1; l >= 0; --l) acc += readlane_v(av[c], l);
            base[c] = acc;
          }
          break;
        }
        if (it >= p.spin) {
          chain_from_seed<T, A, C, F, U, RC>(in, hist, rs, run, tile, lane, p, base);
#ifdef MAVG_AHEAD_STATS
          if (lane == 0) atomicAdd(reinterpret_cast<unsigned int*>(p.stats), 1u);
#endif
          break;
        }
        __builtin_amdgcn_s_sleep(8);
      }
    }
    A lt[C];
#pragma unroll
    for (int c = 0; c < C; ++c) lt[c] = base[c] + (A)dt[c];
    link_store<A, C>(inc, tile, lt, lane);
    if (lane == 0)
#pragma unroll
      for (int c = 0; c < C; ++c) basep[c] = base[c];
  }
  __syncthreads();

  // ---- 5. carry + earlier segments; outputs ----
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
}

}  // namespace mavg
