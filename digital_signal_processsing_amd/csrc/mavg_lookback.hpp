// mavg_lookback.hpp -- the look-ahead scan (ahead_scan_kernel): windows too long for an
// LDS-staged halo, carry from earlier tiles' sums published inside the launch.
#pragma once

#include "mavg_device.hpp"

namespace mavg {

// Accumulator of the in-tile scan: the prefix of d = x - x[n-k] over one
// tile telescopes to two sums of at most T samples, |.| <= 2 * T * 32768 <=
// 2^28 for int16 tiles, so it fits int32 even when the window sum (the
// carry) needs int64 (k > 65535).
template <typename T, typename A> struct ScanAcc { using type = A; };
template <> struct ScanAcc<int16_t, int64_t> { using type = int32_t; };

// Stage the shifted tile [h0, h0 + (U*WG+1)*F) frames in LDS: every lane's
// U units are loaded before any is stored (one memory round trip, not one per
// unit), plus one extra unit for the misaligned x[n-k] read.
template <typename T, int C, int F, int U, int WG, int NT>
__device__ __forceinline__ void stage_shifted_load(const T* __restrict__ in, const T* __restrict__ hist,
                                                   Unit<T, F * C> (&h)[U + 1], long long h0, long long nframes,
                                                   int k, int pre, bool eio, int tid) {
  constexpr int VE = F * C;
  using IO = UnitIO<T, VE>;
  using U_t = Unit<T, VE>;
  const bool fast = h0 >= 0 && h0 + (long long)(U * WG + 1) * F <= nframes;
  auto guarded = [&](int j) {
    U_t r;
    const long long f = h0 + (long long)j * F;
#pragma unroll
    for (int fr = 0; fr < F; ++fr)
#pragma unroll
      for (int c = 0; c < C; ++c) r.e[fr * C + c] = load_elem(in, hist, f + fr, c, C, nframes, k, pre);
    return r;
  };
  if (fast) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      h[u] = IO::template gload<(NT & kNtHalo) != 0>(in + (h0 + (long long)(u * WG + tid) * F) * C, eio);
    if (tid == 0) h[U] = IO::template gload<(NT & kNtHalo) != 0>(in + (h0 + (long long)(U * WG) * F) * C, eio);
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u) h[u] = guarded(u * WG + tid);
    if (tid == 0) h[U] = guarded(U * WG);
  }
}
template <typename T, int C, int F, int U, int WG>
__device__ __forceinline__ void stage_shifted_store(T* stage, const Unit<T, F * C> (&h)[U + 1], int tid) {
  constexpr int VE = F * C;
  using IO = UnitIO<T, VE>;
#pragma unroll
  for (int u = 0; u < U; ++u) IO::store(stage + (u * WG + tid) * VE, h[u]);
  if (tid == 0) IO::store(stage + (U * WG) * VE, h[U]);
}
// Both halves in one call (ORD 0/1).
template <typename T, int C, int F, int U, int WG, int NT>
__device__ __forceinline__ void stage_shifted_tile(const T* __restrict__ in, const T* __restrict__ hist,
                                                   T* stage, long long h0, long long nframes, int k, int pre,
                                                   bool eio, int tid) {
  Unit<T, F * C> h[U + 1];
  stage_shifted_load<T, C, F, U, WG, NT>(in, hist, h, h0, nframes, k, pre, eio, tid);
  stage_shifted_store<T, C, F, U, WG>(stage, h, tid);
}

// ----------------------------------------------------------------------------
// look-ahead scan: the look-back scan in ONE pass over HBM (windows too long
// for an LDS-staged halo)
//
// The carry W[t0-1] needs the sums of the whole tiles inside [t0-k, t0).  The
// two-pass scan streams the signal once more to make them; a one-pass scan in
// which every tile publishes its own sum for later tiles measured 0.15-0.31 of
// peak (tools/tune/onepass_experiment.hpp): the tiles a window reaches back to
// were dispatched only m*8 workgroups earlier (m = k/T), well inside the
// ~2,000 workgroups in flight, so consumers wait on producers that are still
// loading.  Here the workgroup in dispatch slot b publishes the sums of the tile of
// slot b + D ("look-ahead") before it scans its own tile:
//   phase A  every wave loads its share of that tile (default policy, so the
//            lines stay in the XCD's L2 / the MALL) and leaves its partial sum
//            in LDS; after the block's first barrier one wave adds the NW
//            partials in wave order and publishes the tile's record as 8-byte
//            {tag, 32-bit payload} granules with agent-scope (sc1) stores
//            (cdna_hip_programming.md Guideline 16, R2: the data is the flag,
//            no fences); slots b < D publish their own tiles';
//   phase B  the tile scan (as tile_scan_kernel), its whole-tile carry read
//            from the granules with sc1 loads.  The tiles run in remap mode 1
//            (one contiguous run per XCD), so slot b + D is on b's XCD and
//            holds b's tile + D/8: the consumers of a record run >= D slots
//            after its producer, and a tile's own loads hit the lines phase A
//            brought into that XCD's L2.  The first tiles of a run need the
//            records of the previous run's last tiles (dispatched last): the
//            first k/T slots of each run publish those too ("head duty").
// HBM traffic is the algorithmic 8 B/sample (fp32) plus the granules; the
// second read of each tile is served by L2 / MALL.
//
// Round 2 (this form): the shifted tile reaches LDS by LDS-DMA
// (global_load_lds_dwordx4, no staging registers); the partial window (the
// k mod T frames before the window's first whole tile) is summed from the
// x[n-k] units the in-tile scan reads anyway -- they are exactly those frames
// -- instead of an element-wise LDS sweep; the rare paths (head duty, record
// recompute, edge tiles) load one unit at a time so they do not set the
// register allocation (fp32 106 -> 80-90 VGPRs, int16 86-91 -> 69-74); and
// (WREC) each wave publishes its own share of a record as soon as it is
// summed, phase A's loads issued first, so records appear earlier in the
// producer's life and the look-ahead distance can stay short enough for the
// prefetched tiles to survive in the XCD's 4 MB L2.
//
// Progress never depends on scheduling: a granule still untagged after a
// bounded number of polls is recomputed by the waiting wave from the input
// with the producer's lane mapping and order of operations, so the value --
// and the output -- is bitwise the same either way, whatever the dispatch
// order.  The granules are zeroed (hipMemsetAsync) before every launch, so a
// tag is never stale, also under graph replay (Guideline 16, "Re-initialise
// every call").  The carry adds the records in a fixed order: deterministic.
// ----------------------------------------------------------------------------
typedef __attribute__((address_space(1))) unsigned long long gran_t;  // global, never flat
constexpr unsigned long long kGranTag = 1ull << 32;                   // tag 1 in the high word (0 = empty)

// granules per record value: a 32-bit payload each
template <typename SA> struct GranCount { static constexpr int n = sizeof(SA) / 4; };

__device__ __forceinline__ void gran_store(gran_t* g, uint32_t v) {
  __hip_atomic_store(g, kGranTag | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // one sc1 8-B store
}
__device__ __forceinline__ unsigned long long gran_load(const gran_t* g) {
  return __hip_atomic_load(const_cast<gran_t*>(g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1
}
__device__ __forceinline__ uint32_t gran_word(double v, int h) {
  return h == 0 ? (uint32_t)__double2loint(v) : (uint32_t)__double2hiint(v);
}
__device__ __forceinline__ uint32_t gran_word(int32_t v, int) { return (uint32_t)v; }
__device__ __forceinline__ uint32_t gran_word(int64_t v, int h) {
  return h == 0 ? (uint32_t)(uint64_t)v : (uint32_t)((uint64_t)v >> 32);
}
template <typename SA> __device__ __forceinline__ SA gran_value(const uint32_t (&w)[GranCount<SA>::n]);
template <> __device__ __forceinline__ double gran_value<double>(const uint32_t (&w)[2]) {
  return __hiloint2double((int)w[1], (int)w[0]);
}
template <> __device__ __forceinline__ int32_t gran_value<int32_t>(const uint32_t (&w)[1]) { return (int32_t)w[0]; }
template <> __device__ __forceinline__ int64_t gran_value<int64_t>(const uint32_t (&w)[2]) {
  return (int64_t)(((uint64_t)w[1] << 32) | w[0]);
}

// One wave's share of a tile's sum (wave slot wv): lane l sums its units
// u*WG + wv*64 + l over u, frames and channels in order, then one DPP wave
// scan.  A tile's record is its NW shares added in wave order.  Producers
// (phase A), tiles t < D (own registers), head duty and the recompute path
// all run this sequence: bitwise the same value.
template <typename T, typename SA, int C, int F, int U>
__device__ __forceinline__ void wave_record(const Unit<T, F * C> (&x)[U], SA (&r)[C]) {
  SA ls[C];
#pragma unroll
  for (int c = 0; c < C; ++c) ls[c] = (SA)0;
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int fr = 0; fr < F; ++fr)
#pragma unroll
      for (int c = 0; c < C; ++c) ls[c] += to_acc<SA>(x[u].e[fr * C + c]);
#pragma unroll
  for (int c = 0; c < C; ++c) r[c] = readlane(wave_incl_scan(ls[c]), 63);
}

// lanes 0 .. C*NG-1 of the wave each store one granule of tile j's record
template <typename SA, int C>
__device__ __forceinline__ void publish_record(gran_t* gran, long long j, const SA (&r)[C], int lane) {
  constexpr int NG = GranCount<SA>::n;
  MAVG_DCHECK(j >= 0, "record index", j, lane);
  if (lane < C * NG) {
    const int c = lane / NG, h = lane - c * NG;
    SA v = r[0];
#pragma unroll
    for (int i = 1; i < C; ++i)
      if (c == i) v = r[i];
    gran_store(gran + (j * C + c) * NG + h, gran_word(v, h));
  }
}

// The same publication from the NW wave shares of a record in LDS
// (sh[i*C + c], wave i's share of channel c): each publishing lane adds its
// own channel's shares in wave order (the bits of publish_record after the
// same additions) -- an LDS address per lane instead of a register array
// indexed by lane, which the compiler would move to scratch for C >= 4.
template <typename SA, int C, int NW>
__device__ __forceinline__ void publish_record_lds(gran_t* gran, long long j, const SA* sh, int lane) {
  constexpr int NG = GranCount<SA>::n;
  MAVG_DCHECK(j >= 0, "record index", j, lane);
  if (lane < C * NG) {
    const int c = lane / NG, h = lane - c * NG;
    SA v = sh[c];
#pragma unroll
    for (int i = 1; i < NW; ++i) v += sh[i * C + c];
    gran_store(gran + (j * C + c) * NG + h, gran_word(v, h));
  }
}

// first tile of XCD run x under remap mode 1 (remap_tile)
__device__ __forceinline__ long long run_start(unsigned x, unsigned nb) {
  const unsigned q = nb >> 3, r = nb & 7u;
  return (long long)(x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q);
}

// Window-matched runs (launch_ahead_scan, windows past an XCD's L2 reach):
// remap_tile mode G: runs of G consecutive tiles, run r = tiles [rG, rG + G)
// on XCD r mod 8, 8 adjacent runs per period; G ~ k / (8 J T) so that x[n-k]'s
// tile, k/T tiles back, lies J periods back in a run of t's own XCD (read
// J * G of its dispatch slots earlier: an L2 hit); the chip streams one front.
// Blocks past the complete periods map to themselves (remap_tile).
// a wave-uniform 64-bit value computed on the VALU moved to scalar registers,
// so it does not hold two VGPRs across the scan
__device__ __forceinline__ long long uni64(long long v) {
  const int lo = __builtin_amdgcn_readfirstlane((int)(unsigned)(unsigned long long)v);
  const int hi = __builtin_amdgcn_readfirstlane((int)(unsigned)((unsigned long long)v >> 32));
  return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

struct AheadParams {
  const void* in;
  void* out;
  const void* hist;
  long long nframes;
  long long nfull;  // whole tiles (the only ones a carry sums)
  int k;
  int halo_units;   // ceil(k / F): the stage starts halo_units*F frames before the tile
  int xk_off;       // (-k*C) mod VE
  int xcd_remap;    // remap mode (remap_tile): 1, or G (runs of G tiles)
  int ahead;        // D (a multiple of 8): block b publishes the records of block b + D's tile
  int head;         // whole tiles a window can span (k / T): the head duty of remap mode 1
  int spin;         // polls of an untagged granule before recomputing it
  int self;         // self-published records: every tile publishes its own record (no phase A, no
                    // third read), the carry's records are read after the in-tile scan
  int pre;          // frames in front of `in` that are readable signal (load_elem)
  int eio;          // frame-unit launch on element-aligned pointers (UnitIO::gload)
  unsigned long long* gran;  // [nfull][C][NG] granules, zeroed before the launch
  unsigned long long* runs;  // RUNS: [runs_done][C][NGA] run totals, zeroed before the launch
  long long runs_done;       // RUNS: runs [0, runs_done) get a published total
  void* stats;               // MAVG_AHEAD_STATS builds only: {recomputes, polls that waited}
#ifdef MAVG_AHEAD_TRACE
  unsigned long long* trace;  // tuning builds only: [ntiles][8] phase stamps (tools/tune/ahead_trace.py)
#endif
  OutParams o;
};

// wave_record (mavg_lookback.hpp) with one unit in registers at a time: the
// same additions in the same order, so the same bits.  For the rare paths.
template <typename T, typename SA, int C, int F, int U, int WG>
__device__ __forceinline__ void wave_record_lean(const T* __restrict__ in, long long j, int wv, int lane, bool eio,
                                                 SA (&r)[C]) {
  constexpr int VE = F * C;
  constexpr int TF = WG * F * U;
  using IO = UnitIO<T, VE>;
  SA ls[C];
#pragma unroll
  for (int c = 0; c < C; ++c) ls[c] = (SA)0;
#pragma unroll 1
  for (int u = 0; u < U; ++u) {
    const Unit<T, VE> xu = IO::gload(in + (j * TF + (long long)(u * WG + wv * 64 + lane) * F) * C, eio);
#pragma unroll
    for (int fr = 0; fr < F; ++fr)
#pragma unroll
      for (int c = 0; c < C; ++c) ls[c] += to_acc<SA>(xu.e[fr * C + c]);
  }
#pragma unroll
  for (int c = 0; c < C; ++c) r[c] = readlane(wave_incl_scan(ls[c]), 63);
}

// A per-tile record (the NW wave shares added in wave order) from the input,
// one unit in registers at a time: the producer's value, bit for bit.
template <typename T, typename SA, int C, int F, int U, int WG>
__device__ __forceinline__ void tile_record_lean(const T* __restrict__ in, long long j, int lane, bool eio,
                                                 SA (&r)[C]) {
#pragma unroll 1
  for (int wv = 0; wv < WG / 64; ++wv) {
    SA rw[C];
    wave_record_lean<T, SA, C, F, U, WG>(in, j, wv, lane, eio, rw);
#pragma unroll
    for (int c = 0; c < C; ++c) r[c] = wv == 0 ? rw[c] : r[c] + rw[c];
  }
}

// Channel c of a per-tile record (tile_record_lean's value for that channel,
// bit for bit: the same additions in the same order), one accumulator and one
// loaded sample live: the element loads of the rare recompute path set the
// register allocation of the whole kernel otherwise (the wide look-ahead: 8
// fp32 channels, 148 -> 128 VGPRs without a unit-wide load and its select chain).
template <typename T, typename SA, int C, int F, int U, int WG>
__device__ __forceinline__ SA tile_record_chan_lean(const T* __restrict__ in, long long j, int c, int lane) {
  constexpr int TF = WG * F * U;
  SA r = (SA)0;
#pragma unroll 1
  for (int wv = 0; wv < WG / 64; ++wv) {
    SA ls = (SA)0;
#pragma unroll 1
    for (int u = 0; u < U; ++u) {
      const T* px = in + (j * TF + (long long)(u * WG + wv * 64 + lane) * F) * C + c;
#pragma unroll
      for (int fr = 0; fr < F; ++fr) ls += to_acc<SA>(px[fr * C]);
    }
    const SA rw = readlane(wave_incl_scan(ls), 63);
    r = wv == 0 ? rw : r + rw;
  }
  return r;
}

// RUNS: the total of run rr (tiles [rs, rs + G), G <= 64) in A, by one wave:
// lane l takes tile rs + l's per-tile record (its granules, polled like the
// carry's, recomputed from the input when still untagged), then one DPP wave
// scan.  Producers and the consumers' recompute path both run this: the same
// bits whoever computes it.
template <typename T, typename A, int C, int F, int U, int WG>
__device__ __forceinline__ void run_total(const T* __restrict__ in, const gran_t* gran, long long rs, int G,
                                          int spin, int lane, bool eio, A (&tot)[C], void* stats = nullptr) {
  using SA = typename ScanAcc<T, A>::type;
  constexpr int NG = GranCount<SA>::n;
  MAVG_DCHECK(G >= 1 && G <= 64, "run length", G, rs);
  const bool act = lane < G;
  const long long j = rs + lane;
  unsigned long long w[C][NG];
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int h = 0; h < NG; ++h) w[c][h] = act ? gran_load(gran + (j * C + c) * NG + h) : 0ull;
  bool miss = false;
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int h = 0; h < NG; ++h) miss |= act && (w[c][h] >> 32) != 1ull;
#pragma unroll 1
  for (int it = 0; __any(miss) && it < spin; ++it) {
#ifdef MAVG_AHEAD_STATS
    if (lane == 0 && stats != nullptr) atomicAdd(reinterpret_cast<unsigned int*>(stats) + 2, 1u);
#endif
    __builtin_amdgcn_s_sleep(2);
    if (miss) {
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int h = 0; h < NG; ++h) w[c][h] = gran_load(gran + (j * C + c) * NG + h);
    }
    miss = false;
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int h = 0; h < NG; ++h) miss |= act && (w[c][h] >> 32) != 1ull;
  }
  unsigned long long mask = __ballot(miss);
#pragma unroll 1
  while (mask != 0ull) {
    const int l = __builtin_ctzll(mask);
    mask &= mask - 1ull;
    SA r[C];
    tile_record_lean<T, SA, C, F, U, WG>(in, rs + l, lane, eio, r);
    if (lane == l)
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int h = 0; h < NG; ++h) w[c][h] = kGranTag | gran_word(r[c], h);
  }
#pragma unroll
  for (int c = 0; c < C; ++c) {
    uint32_t wd[NG];
#pragma unroll
    for (int h = 0; h < NG; ++h) wd[h] = (uint32_t)w[c][h];
    const A v = act ? (A)gran_value<SA>(wd) : (A)0;
    tot[c] = readlane(wave_incl_scan(v), 63);
  }
}

// RC: keep the own tile's registers (U*F*C samples) across the second barrier
//     and rebuild the in-lane prefix at the output from them and the stage,
//     instead of keeping U*F*C accumulators (fewer registers for fp32, whose
//     accumulators are fp64; the same additions in the same order).
// DMA: stage interior shifted tiles by LDS-DMA (16-B units only).
// DV: the int16 output division (to_out: 0 fp64 product, 1 magic multiply).
// WREC: one record per (tile, wave) instead of per tile, each published by its
//     wave as soon as its share is summed (no barrier before publication; phase
//     A's loads are issued first), so records appear earlier in the producer's
//     life; consumers read NW times as many granules.
// HS: the Hillis-Steele flavour of the in-tile scan (the tile kernel's HS
//     form: the tile is also staged in LDS, lane l holds frames l, l+64, ...
//     of its 64F-frame wave segment, a 6-step DPP log-step scan per register,
//     O(n log n) work); the record carry is the same.  RC must be off (round 5:
//     the log-step scans rebuilt after the carry from the two LDS stages cut the
//     fp32 registers 120 -> 74 and lost, 0.548 -> 0.513 of peak at k=44100, int16
//     mono 0.562 -> 0.517, stereo 0.573 -> 0.527: the scans' VALU no longer hides
//     the record wait; profiles/r05_tuning/hs/).
// RUNS: window-matched runs only (remap mode G, per-tile records): the carry
//     reads the totals of the whole runs inside the window (~8J of them)
//     plus the tile records of the partial runs at its two ends (< 2g),
//     instead of all k/T tile records.  Run rr's total is published by the
//     block that publishes the record of the last tile of run rr + 8 (the
//     same XCD's next run, g slots later, when run rr's records are out).
// MAVG_AHEAD_TRACE (tuning builds only, tools/tune/ahead_trace.py): per tile,
// 100-MHz wall-clock stamps of the phases, taken by thread 0
#ifdef MAVG_AHEAD_TRACE
#define MAVG_ATRACE(slot, v) \
  (p.trace[(unsigned long long)tile * 8 + (slot)] = (unsigned long long)(v))
#define MAVG_ANOW() __builtin_amdgcn_s_memrealtime()
#else
#define MAVG_ATRACE(slot, v) ((void)0)
#define MAVG_ANOW() 0ull
#endif

template <typename T, typename A, int C, int F, int U, int NT, bool RC = false, bool DMA = true, bool WREC = false,
          int DV = 0, bool HS = false, bool RUNS = false, int WG_ = kWG>
__global__ __launch_bounds__(WG_) void ahead_scan_kernel(AheadParams p) {
  static_assert(!(HS && RC), "the Hillis-Steele flavour keeps its per-element prefixes");
  static_assert(!(RUNS && WREC), "run totals sum per-tile records");
  constexpr int WG = WG_;
  constexpr int NW = WG / 64;
  constexpr int VE = F * C;
  constexpr int TF = WG * F * U;
  constexpr int NSEG = U * NW;
  constexpr int kStageUnits = U * WG + 1;
  constexpr int kStageBytes = ((kStageUnits * VE * (int)sizeof(T)) + 15) & ~15;
  using IO = UnitIO<T, VE>;
  using U_t = Unit<T, VE>;
  using SA = typename ScanAcc<T, A>::type;
  constexpr int NG = GranCount<SA>::n;
  constexpr int NGA = GranCount<A>::n;                  // granules of a run total
  constexpr int NGI = RUNS && NGA > NG ? NGA : NG;      // granules of a carry item
  constexpr bool kDma = DMA && IO::kVec && VE * (int)sizeof(T) == 16;

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* stage = reinterpret_cast<T*>(smem);
  A* hsum = reinterpret_cast<A*>(smem + kStageBytes);  // [NW][C] carry partials
  SA* tot = reinterpret_cast<SA*>(hsum + NW * C);       // [NSEG][C] segment totals
  SA* shares = tot + NSEG * C;                           // [3][NW][C] wave shares of the records published here
  // HS: the tile itself, [U*WG] units, after the shares (16-B aligned)
  T* tstage = reinterpret_cast<T*>(smem + ((kStageBytes + (NW * C * (int)sizeof(A)) +
                                            (NSEG + 3 * NW) * C * (int)sizeof(SA) + 15) & ~15));

  const T* __restrict__ in = static_cast<const T*>(p.in);
  T* __restrict__ out = static_cast<T*>(p.out);
  const T* __restrict__ hist = static_cast<const T*>(p.hist);
  gran_t* gran = (gran_t*)p.gran;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int wq = __builtin_amdgcn_readfirstlane(w);
  const int k = p.k;
  const long long nframes = p.nframes;
  const int pre = p.pre;
  const bool eio = F == 1 && p.eio != 0;

  auto map_tile = [&](unsigned b) -> long long { return remap_tile(b, gridDim.x, p.xcd_remap); };
  const long long tile = map_tile(blockIdx.x);
  const long long t0 = tile * TF;
  const int Ha = p.halo_units * F;
  const long long h0 = t0 - Ha;
  MAVG_DCHECK(tile >= 0 && tile < (long long)gridDim.x && t0 < nframes, "ahead tile index", tile, gridDim.x);
  const bool tile_full = (t0 + TF <= nframes);
  if (tid == 0) MAVG_ATRACE(0, MAVG_ANOW());
  const long long a = t0 - k;                                   // first frame of the window before t0
  const long long jlo = a >= 0 ? (a + TF - 1) / TF : 0;         // first whole tile inside it
  constexpr int RPT = WREC ? NW : 1;                            // records per tile
  const long long qlo = jlo * RPT, qhi = tile * RPT;            // records of the whole tiles [jlo, tile)
  const int pcount = a >= 0 ? (int)(jlo * TF - a) : 0;          // window frames before tile jlo (< TF)
  // the carry's items: [0, n1) records qlo + q, [n1, n1 + nR) run totals
  // r1 + q - n1 (RUNS), [n1 + nR, nitem) records rs2 + q - n1 - nR
  long long n1 = qhi - qlo, nR = 0, r1 = 0, rs2 = qhi;
  if constexpr (RUNS) {  // runs of G tiles: [ra1, rb) lie whole inside the window and have totals
    const long long G = p.xcd_remap;
    const long long ra1 = (jlo + G - 1) / G;
    long long rb = tile / G;
    rb = rb < p.runs_done ? rb : p.runs_done;
    if (rb > ra1) {
      n1 = ra1 * G - jlo;
      nR = rb - ra1;
      r1 = ra1;
      rs2 = rb * G;
    }
    n1 = uni64(n1);
    nR = uni64(nR);
    r1 = uni64(r1);
    rs2 = uni64(rs2);
  }
  const long long nitem = n1 + nR + (qhi - rs2);
  auto item_load = [&](long long q, unsigned long long (&v)[C][NGI]) {
    if (RUNS && q >= n1 && q < n1 + nR) {
      const long long r = r1 + (q - n1);
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int h = 0; h < NGI; ++h) v[c][h] = gran_load((const gran_t*)p.runs + (r * C + c) * NGA + h);
    } else {
      const long long j = q < n1 ? qlo + q : rs2 + (q - n1 - nR);
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int h = 0; h < NGI; ++h) v[c][h] = h < NG ? gran_load(gran + (j * C + c) * NG + h) : kGranTag;
    }
  };

  // ---- 1. loads: the tile, the shifted tile, phase A's tile (tile t + D:
  //         default policy, it stays in L2), then the first round of records
  //         (as late as possible: a record read early may not be published yet) ----
  const unsigned nb = gridDim.x;
  const unsigned bd = blockIdx.x + (unsigned)p.ahead;  // the block D dispatch slots later (same XCD)
  const long long ja = bd < nb ? map_tile(bd) : -1;
  const bool produce = !p.self && ja >= 0 && ja < p.nfull;
  U_t xa[U];
  if constexpr (WREC) {  // phase A's loads first: the HBM fetch with the longest latency
    if (produce)
#pragma unroll
      for (int u = 0; u < U; ++u) xa[u] = IO::gload(in + (ja * TF + (long long)(u * WG + tid) * F) * C, eio);
  }
  // HS: whole tiles reach the tile stage by LDS-DMA (no tile registers, no
  // ds_write; the scan reads the stage in its transposed order)
  constexpr bool kHsDma = HS && kDma;
  const bool hs_dma = kHsDma && tile_full && !eio;
  U_t x[U];
  if (hs_dma) {
    if constexpr (kHsDma) {
      unsigned char* tb = reinterpret_cast<unsigned char*>(tstage);
#pragma unroll
      for (int u = 0; u < U; ++u)
        glds16<(NT & kNtLoad) != 0>(in + (t0 + (long long)(u * WG + tid) * F) * C, tb + (u * WG + wq * 64) * 16);
    }
  } else if (tile_full) {
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
  } else if (stage_fast) {  // register staging (units that are not 16 B)
    stage_shifted_tile<T, C, F, U, WG, NT>(in, hist, stage, h0, nframes, k, pre, eio, tid);
  } else {  // edge tiles: guarded, one unit at a time
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
  // a wave's share of a record: kept in LDS for the block's publication
  // after the first barrier, or (WREC) published by the wave itself now
  auto share = [&](int src, long long j, const SA (&r)[C]) {
    if constexpr (WREC) {
      publish_record<SA, C>(gran, j * NW + w, r, lane);
    } else if (lane == 0) {
#pragma unroll
      for (int c = 0; c < C; ++c) shares[(src * NW + w) * C + c] = r[c];
    }
  };
  if (produce) {
    if constexpr (!WREC)
#pragma unroll
      for (int u = 0; u < U; ++u)
        xa[u] = IO::template gload<(NT & kNtPhaseA) != 0>(in + (ja * TF + (long long)(u * WG + tid) * F) * C, eio);
    SA r[C];
    wave_record<T, SA, C, F, U>(xa, r);
    share(0, ja, r);
  }
  if (tid == 0) MAVG_ATRACE(1, MAVG_ANOW());  // phase A summed (and, WREC, published)
  const bool own = (p.self || blockIdx.x < (unsigned)p.ahead) && tile < p.nfull;  // no block D slots earlier
  if (own) {
    SA r[C];
    if (hs_dma) wave_record_lean<T, SA, C, F, U, WG>(in, tile, w, lane, eio, r);  // rare: the first D slots
    else wave_record<T, SA, C, F, U>(x, r);
    share(1, tile, r);
  }
  // head duty (remap mode 1): the first tiles of XCD run x need the records of
  // the last tiles of run x-1, dispatched at the end of the grid; the first
  // `head` blocks of run x publish those
  long long jh = -1;
  if (p.xcd_remap == 1) {
    const unsigned xr = blockIdx.x & 7u, s = blockIdx.x >> 3;
    if (xr >= 1u && s < (unsigned)p.head) {
      const long long j = run_start(xr, nb) - p.head + s;
      if (j >= 0 && j < p.nfull) jh = j;
    }
  }
  if (jh >= 0) {
    SA r[C];
    wave_record_lean<T, SA, C, F, U, WG>(in, jh, w, lane, eio, r);
    share(2, jh, r);
  }
  unsigned long long rv[C][NGI];
  {
    MAVG_DCHECK(qhi <= p.nfull * RPT, "record read range", qhi, p.nfull);
    MAVG_DCHECK(!RUNS || (n1 >= 0 && nR >= 0 && rs2 <= qhi && r1 + nR <= p.runs_done), "carry items", n1, nR);
    if (!p.self && tid < nitem) {
      item_load(tid, rv);
    } else {
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int h = 0; h < NGI; ++h) rv[c][h] = 0ull;
    }
  }
  if constexpr (HS) {
#pragma unroll
    for (int u = 0; u < U && !hs_dma; ++u) IO::store(tstage + (u * WG + tid) * VE, x[u]);
  }
  __syncthreads();
  if (tid == 0) MAVG_ATRACE(2, MAVG_ANOW());  // first barrier
  // publish the records whose wave shares this block holds: wave src adds
  // source src's NW shares in wave order
  if (!WREC && w < 3) {
    const long long j = w == 0 ? (produce ? ja : -1) : (w == 1 ? (own ? tile : -1) : jh);
    if (j >= 0) publish_record_lds<SA, C, NW>(gran, j, shares + (w * NW) * C, lane);
  }
  if constexpr (RUNS) {
    // run totals: wave 3 for the record published from phase A, wave 2 for
    // the block's own; the record's tile is the last of run rr + 8, the same
    // XCD's next run
    if (w >= 2) {
      const long long j = w == 3 ? (produce ? ja : -1) : (own ? tile : -1);
      const long long G = p.xcd_remap;
      if (j >= 0 && (j + 1) % G == 0) {
        const long long rr = (j + 1) / G - 1 - 8;
        if (rr >= 0 && rr < p.runs_done) {
          A tot[C];
          run_total<T, A, C, F, U, WG>(in, gran, rr * G, (int)G, p.spin, lane, eio, tot, p.stats);
#ifdef MAVG_AHEAD_STATS
          if (lane == 0) atomicAdd(reinterpret_cast<unsigned int*>(p.stats) + 3, 1u);
#endif
          if (lane < C * NGA) {
            const int c = lane / NGA, h = lane - c * NGA;
            A v = tot[0];
#pragma unroll
            for (int i = 1; i < C; ++i)
              if (c == i) v = tot[i];
            gran_store((gran_t*)p.runs + (rr * C + c) * NGA + h, gran_word(v, h));
          }
        }
      }
    }
  }

  // ---- 2. the carry's partial window: frames [a, jlo*T), which are the
  //         x[n-k] of this tile's first pcount frames (added in the scan below);
  //         before frame 0 (a < 0): history and/or the peeled head ----
  A hp[C];
#pragma unroll
  for (int c = 0; c < C; ++c) hp[c] = (A)0;
  if (a < 0 && (hist != nullptr || pre > 0)) {
#pragma unroll 1
    for (long long f = a + tid; f < 0; f += WG)
#pragma unroll
      for (int c = 0; c < C; ++c) hp[c] += to_acc<A>(load_elem(in, hist, f, c, C, nframes, k, pre));
  }

  // ---- 3. d = x - x[n-k]; in-lane, wave and segment scans ----
  auto stage_xk = [&](int j) -> U_t {
    const int e = (Ha + j * F - k) * C;  // stage element of x[n-k]
    U_t xk;
    if constexpr (IO::kVec) {
      if (p.xk_off == 0) {
        MAVG_DCHECK(e >= 0 && e + VE <= kStageUnits * VE, "ahead x[n-k] stage index", e, j);
        xk = IO::load(stage + e);
      } else {
        const int e_lo = e - p.xk_off;
        MAVG_DCHECK(e_lo >= 0 && e_lo + 2 * VE <= kStageUnits * VE, "ahead x[n-k] extraction", e_lo, j);
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
    if constexpr (HS) {
      // wave segment u: tile frames sb .. sb + 64F - 1, lane l holds sb + r*64 + l
      const int sb = (u * WG + w * 64) * F;
      SA run[C];
#pragma unroll
      for (int c = 0; c < C; ++c) run[c] = (SA)0;
      // (one scan at a time: the side-by-side scans of the tile kernel's HS form,
      // wave_incl_scan_n, measured 1 % slower here, tools/gpu/r06_dpp_ab.sh)
#pragma unroll
      for (int r = 0; r < F; ++r) {
        const int fl = sb + r * 64 + lane;
#pragma unroll
        for (int c = 0; c < C; ++c) {
          const T xkv = stage[(Ha + fl - k) * C + c];
          if (fl < pcount) hp[c] += to_acc<A>(xkv);  // the partial window: x[n-k] of the first pcount frames
          const SA d = to_acc<SA>(tstage[fl * C + c]) - to_acc<SA>(xkv);
          const SA incl = wave_incl_scan(d);
          v[u][r][c] = incl + run[c];
          run[c] += readlane(incl, 63);
        }
      }
#pragma unroll
      for (int c = 0; c < C; ++c) {
        lx[u][c] = (SA)0;
        if (lane == 0) tot[(u * NW + w) * C + c] = run[c];
      }
      continue;
    }
    const U_t xk = stage_xk(u * WG + tid);
    const int f0 = (u * WG + tid) * F;
    if (f0 + F <= pcount) {
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) hp[c] += to_acc<A>(xk.e[fr * C + c]);
    } else if (f0 < pcount) {
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
        if (f0 + fr < pcount)
#pragma unroll
          for (int c = 0; c < C; ++c) hp[c] += to_acc<A>(xk.e[fr * C + c]);
    }
    SA run[C];
    if constexpr (RC) {
#pragma unroll
      for (int c = 0; c < C; ++c) run[c] = (SA)0;
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) run[c] += to_acc<SA>(x[u].e[fr * C + c]) - to_acc<SA>(xk.e[fr * C + c]);
    } else {
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) {
          const SA d = to_acc<SA>(x[u].e[fr * C + c]) - to_acc<SA>(xk.e[fr * C + c]);
          v[u][fr][c] = fr == 0 ? d : v[u][fr - 1][c] + d;
        }
#pragma unroll
      for (int c = 0; c < C; ++c) run[c] = v[u][F - 1][c];
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const SA incl = wave_incl_scan(run[c]);
      lx[u][c] = incl - run[c];
      const SA segtot = readlane(incl, 63);
      if (lane == 0) tot[(u * NW + w) * C + c] = segtot;
    }
  }

  // ---- 4. whole-tile carry from the records, WG per round ----
  if (tid == 0) MAVG_ATRACE(3, MAVG_ANOW());  // in-tile scan done
  A hq[C];
#pragma unroll
  for (int c = 0; c < C; ++c) hq[c] = (A)0;
#ifdef MAVG_AHEAD_TRACE
  unsigned npoll = 0;  // wave 0's polls of untagged carry items
#endif
#pragma unroll 1
  for (long long qb = 0; qb < nitem; qb += WG) {
    const long long q = qb + tid;
    const bool act = q < nitem;
    if (qb != 0 || p.self) {
      if (act) {
        item_load(q, rv);
      } else {
#pragma unroll
        for (int c = 0; c < C; ++c)
#pragma unroll
          for (int h = 0; h < NGI; ++h) rv[c][h] = 0ull;
      }
    }
    bool miss = false;
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int h = 0; h < NGI; ++h) miss |= act && (rv[c][h] >> 32) != 1ull;
#pragma unroll 1
    for (int it = 0; __any(miss) && it < p.spin; ++it) {
#ifdef MAVG_AHEAD_STATS
      if (lane == 0) atomicAdd(reinterpret_cast<unsigned int*>(p.stats) + 1, 1u);
#endif
#ifdef MAVG_AHEAD_TRACE
      ++npoll;
#endif
      __builtin_amdgcn_s_sleep(2);
      if (miss) item_load(q, rv);
      miss = false;
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int h = 0; h < NGI; ++h) miss |= act && (rv[c][h] >> 32) != 1ull;
    }
    // still untagged: the wave recomputes each such record from the input,
    // with the producer's lane mapping and order of operations
    unsigned long long mask = __ballot(miss);
#pragma unroll 1
    while (mask != 0ull) {
      const int l = __builtin_ctzll(mask);
      mask &= mask - 1ull;
      const long long qq = __shfl(q, l, 64);
      if (RUNS && qq >= n1 && qq < n1 + nR) {  // a run total: the producer's sequence
        const long long G = p.xcd_remap;
        A tot[C];
        run_total<T, A, C, F, U, WG>(in, gran, (r1 + (qq - n1)) * G, (int)G, p.spin, lane, eio, tot);
        if (lane == l)
#pragma unroll
          for (int c = 0; c < C; ++c)
#pragma unroll
            for (int h = 0; h < NGI; ++h) rv[c][h] = kGranTag | gran_word(tot[c], h);
      } else {
        const long long jj = RUNS ? (qq < n1 ? qlo + qq : rs2 + (qq - n1 - nR)) : qlo + qq;
        SA r[C];
        if constexpr (WREC) {  // record jj = (tile, wave)
          wave_record_lean<T, SA, C, F, U, WG>(in, jj / NW, (int)(jj % NW), lane, eio, r);
        } else {
          tile_record_lean<T, SA, C, F, U, WG>(in, jj, lane, eio, r);
        }
        if (lane == l)
#pragma unroll
          for (int c = 0; c < C; ++c)
#pragma unroll
            for (int h = 0; h < NGI; ++h) rv[c][h] = kGranTag | (h < NG ? gran_word(r[c], h) : 0u);
      }
#ifdef MAVG_AHEAD_STATS
      if (lane == 0) atomicAdd(reinterpret_cast<unsigned int*>(p.stats), 1u);
#endif
    }
    if (act) {
      const bool run_item = RUNS && q >= n1 && q < n1 + nR;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        if constexpr (RUNS && NGA > NG) {
          uint32_t wa[NGA], ws[NG];
#pragma unroll
          for (int h = 0; h < NGA; ++h) wa[h] = (uint32_t)rv[c][h];
#pragma unroll
          for (int h = 0; h < NG; ++h) ws[h] = (uint32_t)rv[c][h];
          hq[c] += run_item ? gran_value<A>(wa) : (A)gran_value<SA>(ws);
        } else if constexpr (RUNS) {  // NGA == NG
          uint32_t wd[NGI];
#pragma unroll
          for (int h = 0; h < NGI; ++h) wd[h] = (uint32_t)rv[c][h];
          hq[c] += run_item ? gran_value<A>(wd) : (A)gran_value<SA>(wd);
        } else {
          uint32_t wd[NG];
#pragma unroll
          for (int h = 0; h < NG; ++h) wd[h] = (uint32_t)rv[c][h];
          hq[c] += (A)gran_value<SA>(wd);
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const A r = readlane(wave_incl_scan(hp[c] + hq[c]), 63);
    if (lane == 0) hsum[w * C + c] = r;
  }
  if (tid == 0) MAVG_ATRACE(4, MAVG_ANOW());  // wave 0's carry items read
  __syncthreads();
  if (tid == 0) MAVG_ATRACE(5, MAVG_ANOW());  // second barrier

  // ---- 5. carry + earlier segments; outputs ----
  static_assert(NSEG <= 64, "segment totals are scanned across one wave");
  A w0[C];
  SA ex[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    w0[c] = (A)0;
#pragma unroll
    for (int i = 0; i < NW; ++i) w0[c] += hsum[i * C + c];
    const SA tv = lane < NSEG ? tot[lane * C + c] : (SA)0;
    ex[c] = wave_incl_scan(tv) - tv;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if constexpr (HS) {
      const long long sb = t0 + (long long)(u * WG + w * 64) * F;
      A b[C];
#pragma unroll
      for (int c = 0; c < C; ++c) b[c] = w0[c] + (A)readlane(ex[c], u * NW + wq);
#pragma unroll
      for (int r = 0; r < F; ++r) {
        const long long f = sb + r * 64 + lane;
        if (tile_full || f < nframes)
#pragma unroll
          for (int c = 0; c < C; ++c) {
            const T yv = to_out<T, A, DV>(b[c] + (A)v[u][r][c], p.o);
            if constexpr ((NT & kNtStore) != 0) __builtin_nontemporal_store(yv, out + f * C + c);
            else out[f * C + c] = yv;
          }
      }
      continue;
    }
    const long long f = t0 + (long long)(u * WG + tid) * F;
    A b[C];
#pragma unroll
    for (int c = 0; c < C; ++c) b[c] = w0[c] + (A)(readlane(ex[c], u * NW + wq) + lx[u][c]);
    U_t y;
    if constexpr (RC) {
      const U_t xk = stage_xk(u * WG + tid);
      SA run[C];
#pragma unroll
      for (int c = 0; c < C; ++c) run[c] = (SA)0;
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) {
          run[c] += to_acc<SA>(x[u].e[fr * C + c]) - to_acc<SA>(xk.e[fr * C + c]);
          y.e[fr * C + c] = to_out<T, A, DV>(b[c] + (A)run[c], p.o);
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
#ifdef MAVG_AHEAD_TRACE
  if (tid == 0) {
    MAVG_ATRACE(6, MAVG_ANOW());  // outputs issued
    MAVG_ATRACE(7, (unsigned long long)npoll);
  }
#endif
}

}  // namespace mavg
