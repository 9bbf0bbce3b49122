// onepass_experiment.hpp -- a one-pass look-back scan (onepass_scan_kernel),
// kept as a measured experiment for tools/tune/tune_scan.hip only; NOT part of
// libmavg.  Measured 0.15-0.38 of HBM peak with zero record recomputes against
// 0.48-0.53 for the two-pass look-back it would replace (DESIGN.md "Tuning",
// profiles/r01_tuning/onepass/): the device-scope record traffic (stores
// written through past the XCD's L2, loads that bypass it) lengthens every
// tile's lifetime by memory round trips the two-pass scan does not pay.
#pragma once

#include "../../digital_signal_processsing_amd/csrc/mavg_launch.hpp"

namespace mavg {

// ----------------------------------------------------------------------------
// One-pass look-back scan (windows too long for an LDS-staged halo)
//
// The same flat, XCD-remapped tiles and shifted-tile stage as
// lookback_scan_kernel, but without pass 1: every wave publishes the sum of
// its part of its tile ("record", one 64-bit word per (tile, wave, channel))
// as soon as its tile has arrived in registers, and a tile takes the
// whole-tile part of its carry W[t0-1] from the records of the tiles inside
// [t0-k, t0).  Those tiles lie k frames back: all but the last few finished
// long ago.  The record loads are issued before the shifted tile is staged
// and checked only after the in-tile scan, so a wait, if any, overlaps the
// tile's own work.
//
// Visibility: records are written and read with agent-scope relaxed atomics
// (write-through / bypass of the XCD's L2), each record is one atomic word,
// and the slots are filled with a sentinel by reset_records_kernel before the
// launch, so no fences or flags are needed.
//
// Progress never depends on scheduling: a record still empty after a bounded
// wait is recomputed by the waiting wave itself, from the input, with the
// producer's lane mapping and order of operations, so the value (and the
// output) is bitwise the same either way and the launch cannot deadlock
// whatever order the workgroups are dispatched in.  Recomputations are
// counted in the workspace header (printed by tune_scan).
//
// The carry sums the records in a fixed order, so results are deterministic
// (fp32: fp64 sums whose association depends only on n, k and the tile shape).
// ----------------------------------------------------------------------------
constexpr unsigned long long kRecEmpty = 0x7FF7FFF77FF7FFF7ull;  // a NaN payload; no int tile sum reaches it
constexpr int kOnepassSpin = 4096;   // polls before recomputing (each >= one trip past L2 + s_sleep)

__device__ __forceinline__ unsigned long long rec_pack(double v) { return (unsigned long long)__double_as_longlong(v); }
__device__ __forceinline__ unsigned long long rec_pack(int32_t v) { return (unsigned long long)(long long)v; }
template <typename SA> __device__ __forceinline__ SA rec_unpack(unsigned long long r);
template <> __device__ __forceinline__ double rec_unpack<double>(unsigned long long r) {
  return __longlong_as_double((long long)r);
}
template <> __device__ __forceinline__ int32_t rec_unpack<int32_t>(unsigned long long r) { return (int32_t)(long long)r; }

__device__ __forceinline__ void rec_store(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long rec_load(const unsigned long long* p) {
  return __hip_atomic_load(const_cast<unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename R = unsigned long long>  // a template: one definition across the per-family TUs
__global__ void reset_records_kernel(R* __restrict__ rec, long long n, unsigned int* __restrict__ fallbacks) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *fallbacks = 0u;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    rec[i] = (R)kRecEmpty;
}

// One wave's record values for tile j, wave slot wv: lane l sums units
// u*WG + wv*64 + l over u and frames in order, then one DPP wave scan.  The
// producer (on its registers) and the recompute path (from memory) run this
// same sequence, so both give the same bits.
template <typename T, typename SA, int C, int F, int U, int WG>
__device__ __forceinline__ void wave_record_values(const Unit<T, F * C> (&x)[U], SA (&r)[C]) {
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

struct OnepassParams {
  const void* in;
  void* out;
  const void* hist;
  long long nframes;
  int k;
  int halo_units;   // ceil(k / F): the stage starts halo_units*F frames before the tile
  int xk_off;       // (-k*C) mod VE
  int xcd_remap;    // remap mode (remap_tile)
  unsigned long long* rec;        // [ntiles][NW][C] records (sentinel-filled)
  unsigned int* fallbacks;        // recompute counter (workspace header)
  OutParams o;
};

template <typename T, typename A, int C, int F, int U, int NT>
__global__ __launch_bounds__(kWG) void onepass_scan_kernel(OnepassParams p) {
  constexpr int WG = kWG;
  constexpr int NW = WG / 64;
  constexpr int VE = F * C;
  constexpr int TF = WG * F * U;
  constexpr int NSEG = U * NW;
  constexpr int kStageUnits = U * WG + 1;  // the shifted tile + one unit for the misaligned x[n-k] read
  constexpr int kStageBytes = ((kStageUnits * VE * (int)sizeof(T)) + 15) & ~15;
  using IO = UnitIO<T, VE>;
  using U_t = Unit<T, VE>;
  using SA = typename ScanAcc<T, A>::type;  // in-tile scan and records; the carry stays in A

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* stage = reinterpret_cast<T*>(smem);
  A* hsum = reinterpret_cast<A*>(smem + kStageBytes);  // [NW][C] carry partials
  SA* tot = reinterpret_cast<SA*>(hsum + NW * C);       // [NSEG][C] segment totals

  const T* __restrict__ in = static_cast<const T*>(p.in);
  T* __restrict__ out = static_cast<T*>(p.out);
  const T* __restrict__ hist = static_cast<const T*>(p.hist);
  unsigned long long* rec = p.rec;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int k = p.k;
  const long long nframes = p.nframes;

  const long long tile = remap_tile(blockIdx.x, gridDim.x, p.xcd_remap);
  const long long t0 = tile * TF;
  const int Ha = p.halo_units * F;
  const long long h0 = t0 - Ha;
  const bool tile_full = (t0 + TF <= nframes);
  const long long a = t0 - k;
  const long long jlo = a >= 0 ? (a + TF - 1) / TF : 0;
  // records of the whole tiles [jlo, tile): q = j*NW + wave slot in [qlo, qhi)
  const long long qlo = jlo * NW, qhi = tile * NW;

  // ---- tile -> registers ----
  U_t x[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long f = t0 + (long long)(u * WG + tid) * F;
    if (tile_full) {
      x[u] = IO::template load<(NT & kNtLoad) != 0>(in + f * C);
    } else {
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) x[u].e[fr * C + c] = load_elem(in, hist, f + fr, c, C, nframes, k);
    }
  }
  // ---- shifted tile [h0, h0 + kStageUnits*F) -> LDS (k frames back: L2 /
  //      MALL); the first round of record loads is issued after it so that
  //      the stage stores do not wait for them (checked after the in-tile scan) ----
  stage_shifted_tile<T, C, F, U, WG, NT>(in, hist, stage, h0, nframes, k, tid);
  // publish this wave's record after the stage loads are in flight: a store
  // issued earlier would make them wait for its write-through to complete
  if (tile_full) {  // every tile a later window can contain whole is full
    SA r[C];
    wave_record_values<T, SA, C, F, U, WG>(x, r);
    if (lane == 0)
#pragma unroll
      for (int c = 0; c < C; ++c) rec_store(&rec[(tile * NW + w) * C + c], rec_pack(r[c]));
  }
  unsigned long long rv[C];
  {
    const long long q = qlo + tid;
#pragma unroll
    for (int c = 0; c < C; ++c) rv[c] = q < qhi ? rec_load(&rec[q * C + c]) : 0ull;
  }
  __syncthreads();

  // ---- partial carry: the part of [a, t0) before the first whole tile ----
  A hp[C];
#pragma unroll
  for (int c = 0; c < C; ++c) hp[c] = (A)0;
  if (a >= 0) {
    const int pcount = (int)(jlo * TF - a);  // < TF frames, inside the stage
    const int s0 = Ha - k;                   // stage frame of a
    for (int i = tid; i < pcount; i += WG)
#pragma unroll
      for (int c = 0; c < C; ++c) hp[c] += to_acc<A>(stage[(s0 + i) * C + c]);
  } else if (hist != nullptr) {
    for (long long f = a + tid; f < 0; f += WG)
#pragma unroll
      for (int c = 0; c < C; ++c) hp[c] += to_acc<A>(load_elem(in, hist, f, c, C, nframes, k));
  }

  // ---- d = x - x[n-k]; in-lane, wave and segment scans ----
  SA v[U][F][C];
  SA lx[U][C];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int j = u * WG + tid;
    const int e = (Ha + j * F - k) * C;
    U_t xk;
    if constexpr (IO::kVec) {
      if (p.xk_off == 0) {
        xk = IO::load(stage + e);
      } else {
        const int e_lo = e - p.xk_off;
        U_t a0 = IO::load(stage + e_lo);
        U_t a1 = IO::load(stage + e_lo + VE);
        xk = extract(a0, a1, p.xk_off);
      }
    } else {
#pragma unroll
      for (int i = 0; i < VE; ++i) xk.e[i] = stage[e + i];
    }
#pragma unroll
    for (int fr = 0; fr < F; ++fr)
#pragma unroll
      for (int c = 0; c < C; ++c) v[u][fr][c] = to_acc<SA>(x[u].e[fr * C + c]) - to_acc<SA>(xk.e[fr * C + c]);
#pragma unroll
    for (int fr = 1; fr < F; ++fr)
#pragma unroll
      for (int c = 0; c < C; ++c) v[u][fr][c] += v[u][fr - 1][c];
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const SA t = v[u][F - 1][c];
      const SA incl = wave_incl_scan(t);
      lx[u][c] = incl - t;
      const SA segtot = readlane(incl, 63);
      if (lane == 0) tot[(u * NW + w) * C + c] = segtot;
    }
  }

  // ---- whole-tile carry from the records (wave-uniform rounds of WG records) ----
  A hq[C];
#pragma unroll
  for (int c = 0; c < C; ++c) hq[c] = (A)0;
  for (long long qb = qlo; qb < qhi; qb += WG) {
    const long long q = qb + tid;
    const bool act = q < qhi;
    if (qb != qlo) {
#pragma unroll
      for (int c = 0; c < C; ++c) rv[c] = act ? rec_load(&rec[q * C + c]) : 0ull;
    }
    for (int it = 0;; ++it) {
      bool miss = false;
#pragma unroll
      for (int c = 0; c < C; ++c) miss |= act && rv[c] == kRecEmpty;
      if (!__any(miss) || it == kOnepassSpin) break;
      __builtin_amdgcn_s_sleep(4);
      if (miss)
#pragma unroll
        for (int c = 0; c < C; ++c) rv[c] = rec_load(&rec[q * C + c]);
    }
    // still empty: the wave recomputes each missing record itself
    bool miss = false;
#pragma unroll
    for (int c = 0; c < C; ++c) miss |= act && rv[c] == kRecEmpty;
    unsigned long long mask = __ballot(miss);
    while (mask != 0ull) {
      const int l = __builtin_ctzll(mask);
      mask &= mask - 1ull;
      const long long qq = __shfl(q, l, 64);
      const long long jj = qq / NW;
      const int wv = (int)(qq - jj * NW);
      U_t xr[U];
#pragma unroll
      for (int u = 0; u < U; ++u) xr[u] = IO::load(in + (jj * TF + (long long)(u * WG + wv * 64 + lane) * F) * C);
      SA r[C];
      wave_record_values<T, SA, C, F, U, WG>(xr, r);
      if (lane == l)
#pragma unroll
        for (int c = 0; c < C; ++c) rv[c] = rec_pack(r[c]);
      if (lane == 0) atomicAdd(p.fallbacks, 1u);
    }
    if (act)
#pragma unroll
      for (int c = 0; c < C; ++c) hq[c] += (A)rec_unpack<SA>(rv[c]);
  }
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const A r = readlane(wave_incl_scan(hp[c] + hq[c]), 63);
    if (lane == 0) hsum[w * C + c] = r;
  }
  __syncthreads();

  // ---- carry + earlier segments; outputs ----
  static_assert(NSEG <= 64, "segment totals are scanned across one wave");
  const int wu = __builtin_amdgcn_readfirstlane(w);
  A base[U][C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    A w0 = (A)0;
#pragma unroll
    for (int i = 0; i < NW; ++i) w0 += hsum[i * C + c];
    const SA tv = lane < NSEG ? tot[lane * C + c] : (SA)0;
    const SA ex = wave_incl_scan(tv) - tv;
#pragma unroll
    for (int u = 0; u < U; ++u) base[u][c] = w0 + (A)readlane(ex, u * NW + wu);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long f = t0 + (long long)(u * WG + tid) * F;
    U_t y;
#pragma unroll
    for (int fr = 0; fr < F; ++fr)
#pragma unroll
      for (int c = 0; c < C; ++c) y.e[fr * C + c] = to_out<T, A>(base[u][c] + (A)(lx[u][c] + v[u][fr][c]), p.o);
    if (tile_full) {
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

// one-pass look-back scan: reset the record slots, then one scan launch
// whose tiles publish per-wave tile sums and take their carry from earlier
// tiles' records (mavg_onepass.hpp).  Workspace: header + one 64-bit record
// per (whole tile, wave, channel).
template <typename T, typename A, int C, int F, int U, int NT = 0>
int launch_onepass_scan(const void* in, void* out, const void* hist, long long nframes, int k, hipStream_t st,
                        Workspace ws, int xcd_remap = kRemapGroup) {
  constexpr int TF = kWG * F * U;
  constexpr int VE = F * C;
  constexpr int NSEG = U * kNW;
  constexpr size_t kStageBytes = (((size_t)(U * kWG + 1) * VE * sizeof(T)) + 15) & ~(size_t)15;
  const long long ntiles = (nframes + TF - 1) / TF;
  const long long nfull = nframes / TF;
  if (ntiles > 0x7fffffffLL) return MAVG_ERR_UNSUPPORTED;
  const long long nrec = std::max<long long>(nfull, 1) * kNW * C;
  const size_t need = (size_t)kLookbackHeader + (size_t)nrec * sizeof(unsigned long long);
  const size_t lds = kStageBytes + (size_t)(NSEG + kNW) * C * sizeof(A);
  if (lds > kLdsBudget) return MAVG_ERR_UNSUPPORTED;
  if (g_plan) {
    snprintf(g_plan->text, sizeof(g_plan->text),
             "onepass_scan<%s,acc=%s,C=%d,F=%d,U=%d,nt=%d> grid=%lld block=%d lds=%zu tile_frames=%d "
             "remap=%d ws=%zu",
             type_name<T>(), type_name<A>(), C, F, U, NT, ntiles, kWG, lds, TF, xcd_remap, need);
    g_plan->ws_bytes = need;
    return MAVG_OK;
  }
  if (ws.ptr == nullptr || ws.bytes < need) return MAVG_ERR_WORKSPACE;
  if ((reinterpret_cast<uintptr_t>(ws.ptr) & 7u) != 0) return MAVG_ERR_MISALIGNED;
  unsigned int* fb = static_cast<unsigned int*>(ws.ptr);
  unsigned long long* rec =
      reinterpret_cast<unsigned long long*>(static_cast<unsigned char*>(ws.ptr) + kLookbackHeader);
  const long long rgrid = std::min<long long>((nrec + 255) / 256, 2048);
  hipLaunchKernelGGL(reset_records_kernel<unsigned long long>, dim3((unsigned)rgrid), dim3(256), 0, st, rec, nrec, fb);
  OnepassParams p{};
  p.in = in;
  p.out = out;
  p.hist = hist;
  p.nframes = nframes;
  p.k = k;
  p.o = make_out_params(k);
  p.halo_units = (k + F - 1) / F;
  p.xk_off = (int)((VE - ((long long)k * C) % VE) % VE);
  p.xcd_remap = xcd_remap;
  p.rec = rec;
  p.fallbacks = fb;
  hipLaunchKernelGGL((onepass_scan_kernel<T, A, C, F, U, NT>), dim3((unsigned)ntiles), dim3(kWG), lds, st, p);
  return hipGetLastError() == hipSuccess ? MAVG_OK : MAVG_ERR_HIP;
}

}  // namespace mavg
