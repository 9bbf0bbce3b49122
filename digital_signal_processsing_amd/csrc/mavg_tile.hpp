// mavg_tile.hpp -- the flat-tile scan (tile_scan_kernel): Blelloch and Hillis-Steele
// flavours.
#pragma once

#include "mavg_device.hpp"

namespace mavg {

// ----------------------------------------------------------------------------
// flat-tile scan kernel: one short-lived workgroup per tile of T = 256*F*U
// frames.  The carry into the tile is rebuilt from its k-frame halo instead
// of being chained between workgroups:
//     W[t0-1] = sum_{j=t0-k}^{t0-1} x[j]            (halo reduction)
//     W[n]    = W[t0-1] + scan_{t0..n}(x[m] - x[m-k])
// The halo and the tile are staged in LDS (x[n-k] reads).  Workgroups are
// remapped so that consecutive tiles run on the same XCD: the halo is the
// tail of the tile that XCD just read, an L2 hit, and all concurrently
// running workgroups of an XCD touch one contiguous window of HBM (row-buffer
// locality: the "flat" access shape that reaches 82% of HBM peak for a copy,
// tools/tune/membw.hip).  Two barriers per workgroup; no inter-workgroup
// communication.  (Reading x[n-k] and the halo from global memory instead of
// LDS measured 5.1 vs 6.26 TB/s, profiles/r01_tuning.)
// ----------------------------------------------------------------------------
struct TileParams {
  const void* in;
  void* out;
  const void* hist;
  long long nframes;
  long long ntiles;
  int k;
  int halo_units;  // ceil(k / F): units staged before the tile
  int xk_off;      // (-k*C) mod VE
  int xcd_remap;   // remap mode (remap_tile): 0 identity, 1 contiguous per XCD, G>1 grouped
  int pre;         // frames in front of `in` that are readable signal (load_elem)
  int eio;         // frame-unit launch on element-aligned pointers (UnitIO::gload)
  OutParams o;
};

// HS: Hillis-Steele flavour.  Transposed ownership: lane l holds frames l,
//     l+64, ..., l+64(F-1) of its 64F-frame wave segment, so every register
//     holds 64 consecutive frames and the log-step scan runs on DPP (6 steps
//     per element, O(n log n) work) with a scalar carry across the F registers.
// NT: bit 0 non-temporal output stores, bit 1 non-temporal input loads,
//     bit 2 (kNtSplit) non-temporal tile loads except the last halo-size
//     frames, bit 3 (kNtHalo) non-temporal halo loads.
// RC (Blelloch flavour): keep only each lane's total across the second
//     barrier and rebuild the in-lane prefix afterwards from the LDS stage
//     (the tile and x[n-k] are both staged), in the same order, so the
//     outputs are bitwise the same with U*F*C fewer live accumulators.
// DMA (Blelloch flavour, 16-B units): interior tiles stage the halo and the
//     tile in LDS by LDS-DMA (global_load_lds_dwordx4, no staging registers,
//     no ds_write) and the scan reads x from the stage.
template <typename T, typename A, int C, int F, int U, bool HS, int NT = kNtLoad | kNtStore, int WG = kWG,
          bool RC = true, int DV = 0, bool DMA = false>
__global__ __launch_bounds__(WG) void tile_scan_kernel(TileParams p) {
  constexpr int NW = WG / 64;
  constexpr int VE = F * C;
  constexpr int TF = WG * F * U;           // tile frames
  constexpr int NSEG = U * NW;
  constexpr bool kRC = RC && !HS;
  using IO = UnitIO<T, VE>;
  using U_t = Unit<T, VE>;

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int Hu = p.halo_units;
  const int Ha = Hu * F;                     // staged halo frames (>= k)
  const int stage_bytes = (((Hu + U * WG + 1) * VE * (int)sizeof(T)) + 15) & ~15;
  T* stage = reinterpret_cast<T*>(smem);     // [Hu + U*256 + 1 pad] units
  A* tot = reinterpret_cast<A*>(smem + stage_bytes);  // [NSEG][C] segment totals
  A* hsum = tot + NSEG * C;                            // [NW][C] halo partial sums

  const T* __restrict__ in = static_cast<const T*>(p.in);
  T* __restrict__ out = static_cast<T*>(p.out);
  const T* __restrict__ hist = static_cast<const T*>(p.hist);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int k = p.k;
  const long long nframes = p.nframes;
  const int pre = p.pre;
  const bool eio = F == 1 && p.eio != 0;

  // bijective XCD-aware remap (cdna_hip_programming.md 5.5 T1): blocks b and
  // b+8 share an XCD; give each XCD a contiguous run of tiles.
  const long long tile = remap_tile(blockIdx.x, gridDim.x, p.xcd_remap);
  const long long t0 = tile * TF;
  const long long h0 = t0 - Ha;              // first staged halo frame
  MAVG_DCHECK(tile >= 0 && tile < p.ntiles && t0 < nframes, "tile index", tile, p.ntiles);
  MAVG_DCHECK(stage_bytes + (NSEG + NW) * C * (int)sizeof(A) <= (int)(WG >= 1024 ? 80 * 1024 : 64 * 1024),
              "tile LDS layout", stage_bytes, Hu);
  const bool tile_full = (t0 + TF <= nframes);

  constexpr bool kDma = DMA && !HS && IO::kVec && VE * (int)sizeof(T) == 16;
  const bool dma = kDma && tile_full && h0 >= 0 && !eio;  // uniform
  constexpr bool kXs = kRC || kDma;  // x read back from the stage
  // ---- tile -> registers -> LDS (or straight to LDS by LDS-DMA) ----
  U_t x[U];
  if constexpr (kDma) {
    if (dma) {
      const int wq = __builtin_amdgcn_readfirstlane(w);
      unsigned char* sb = reinterpret_cast<unsigned char*>(stage);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long f = t0 + (long long)(u * WG + tid) * F;
        unsigned char* d = sb + (Hu + u * WG + wq * 64) * 16;
        if constexpr ((NT & kNtSplit) != 0) {
          // frames the next tile's halo re-reads keep the default policy (L2)
          if ((u * WG + tid) * F + F > TF - Ha) glds16<false>(in + f * C, d);
          else glds16<true>(in + f * C, d);
        } else {
          glds16<(NT & kNtLoad) != 0>(in + f * C, d);
        }
      }
      for (int j0 = 0; j0 < Hu; j0 += WG) {
        const int j = j0 + tid;
        if (j < Hu) glds16<(NT & kNtHalo) != 0>(in + (h0 + (long long)j * F) * C, sb + (j0 + wq * 64) * 16);
      }
      if (tid == 0) {
        U_t z;
#pragma unroll
        for (int i = 0; i < VE; ++i) z.e[i] = (T)0;
        IO::store(stage + (Hu + U * WG) * VE, z);
      }
    }
  }
#pragma unroll
  for (int u = 0; u < U && !dma; ++u) {
    const long long f = t0 + (long long)(u * WG + tid) * F;
    if (tile_full) {
      if constexpr ((NT & kNtSplit) != 0) {
        // frames the next tile's halo re-reads keep the default policy (L2)
        if ((u * WG + tid) * F + F > TF - Ha) x[u] = IO::template gload<false>(in + f * C, eio);
        else x[u] = IO::template gload<true>(in + f * C, eio);
      } else {
        x[u] = IO::template gload<(NT & kNtLoad) != 0>(in + f * C, eio);
      }
    } else {
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) x[u].e[fr * C + c] = load_elem(in, hist, f + fr, c, C, nframes, k, pre);
    }
  }
  // ---- halo -> LDS (re-read of the previous tile's tail: L2) ----
  if (!dma) {
    const bool halo_fast = h0 >= 0;
    for (int j = tid; j < Hu; j += WG) {
      const long long f = h0 + (long long)j * F;
      U_t h;
      if (halo_fast) {
        h = IO::template gload<(NT & kNtHalo) != 0>(in + f * C, eio);
      } else {
#pragma unroll
        for (int fr = 0; fr < F; ++fr)
#pragma unroll
          for (int c = 0; c < C; ++c) h.e[fr * C + c] = load_elem(in, hist, f + fr, c, C, nframes, k, pre);
      }
      IO::store(stage + j * VE, h);
    }
  }
  if (!dma) {
#pragma unroll
    for (int u = 0; u < U; ++u) IO::store(stage + (Hu + u * WG + tid) * VE, x[u]);
    if (tid == 0) {
      U_t z;
#pragma unroll
      for (int i = 0; i < VE; ++i) z.e[i] = (T)0;
      IO::store(stage + (Hu + U * WG) * VE, z);   // pad unit (k < F reads one unit past the tile)
    }
  }
  __syncthreads();

  // ---- halo reduction: W[t0-1] = sum of the k frames before t0 ----
  {
    A hs[C];
#pragma unroll
    for (int c = 0; c < C; ++c) hs[c] = (A)0;
    for (int i = Ha - k + tid; i < Ha; i += WG)
#pragma unroll
      for (int c = 0; c < C; ++c) hs[c] += to_acc<A>(stage[i * C + c]);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const A r = readlane(wave_incl_scan(hs[c]), 63);
      if (lane == 0) hsum[w * C + c] = r;
    }
  }

  // x[n-k] for lane unit j, from the LDS stage (an unaligned x[n-k]: two
  // aligned units and a uniform shift)
  auto stage_xk = [&](int j) -> U_t {
    const int e = (Ha + j * F - k) * C;
    U_t xk;
    if constexpr (IO::kVec) {
      if (p.xk_off == 0) {
        MAVG_DCHECK(e >= 0 && e + VE <= (Hu + U * WG + 1) * VE, "tile x[n-k] stage index", e, j);
        xk = IO::load(stage + e);
      } else {
        const int e_lo = e - p.xk_off;
        MAVG_DCHECK(e_lo >= 0 && e_lo + 2 * VE <= (Hu + U * WG + 1) * VE, "tile x[n-k] extraction", e_lo, j);
        U_t a = IO::load_whole(stage + e_lo);
        U_t b = IO::load_whole(stage + e_lo + VE);
        xk = extract(a, b, p.xk_off);
      }
    } else {
#pragma unroll
      for (int i = 0; i < VE; ++i) xk.e[i] = stage[e + i];
    }
    return xk;
  };

  // ---- d = x - x[n-k]; in-lane, wave and segment scans ----
  A v[kRC ? 1 : U][F][C];  // in-lane prefixes (Blelloch without RC) / wave scans (HS)
  A lx[U][C];              // exclusive prefix of the lane totals inside the wave
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if constexpr (HS) {
      const int sb = (u * WG + w * 64) * F;  // tile-local first frame of this wave segment
      A run[C];
#pragma unroll
      for (int c = 0; c < C; ++c) run[c] = (A)0;
      // the F*C log-step scans of the segment side by side (wave_incl_scan_n), then the
      // carries across the F registers in register order
      A incl[F * C];
#pragma unroll
      for (int r = 0; r < F; ++r) {
        const int fl = sb + r * 64 + lane;
#pragma unroll
        for (int c = 0; c < C; ++c)
          incl[r * C + c] = to_acc<A>(stage[(Ha + fl) * C + c]) - to_acc<A>(stage[(Ha + fl - k) * C + c]);
      }
      wave_incl_scan_n(incl);
#pragma unroll
      for (int r = 0; r < F; ++r)
#pragma unroll
        for (int c = 0; c < C; ++c) {
          v[u][r][c] = incl[r * C + c] + run[c];
          run[c] += readlane(incl[r * C + c], 63);
        }
#pragma unroll
      for (int c = 0; c < C; ++c) {
        lx[u][c] = (A)0;
        if (lane == 0) tot[(u * NW + w) * C + c] = run[c];
      }
    } else {
      const int j = u * WG + tid;
      const U_t xk = stage_xk(j);
      A run[C];
      if constexpr (kRC) {
        const U_t xu = IO::load(stage + (Hu + j) * VE);  // x's registers died at the stage store
#pragma unroll
        for (int c = 0; c < C; ++c) run[c] = (A)0;
#pragma unroll
        for (int fr = 0; fr < F; ++fr)
#pragma unroll
          for (int c = 0; c < C; ++c) run[c] += to_acc<A>(xu.e[fr * C + c]) - to_acc<A>(xk.e[fr * C + c]);
      } else {
        U_t xu;
        if constexpr (kXs) xu = IO::load(stage + (Hu + j) * VE);
        else xu = x[u];
#pragma unroll
        for (int fr = 0; fr < F; ++fr)
#pragma unroll
          for (int c = 0; c < C; ++c) {
            const A d = to_acc<A>(xu.e[fr * C + c]) - to_acc<A>(xk.e[fr * C + c]);
            v[u][fr][c] = fr == 0 ? d : v[u][fr - 1][c] + d;
          }
#pragma unroll
        for (int c = 0; c < C; ++c) run[c] = v[u][F - 1][c];
      }
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const A incl = wave_incl_scan(run[c]);
        lx[u][c] = incl - run[c];
        const A segtot = readlane(incl, 63);
        if (lane == 0) tot[(u * NW + w) * C + c] = segtot;
      }
    }
  }
  __syncthreads();

  // ---- carry: halo sum + earlier segments; outputs ----
  // segment s = u*NW + w needs the sum of the totals of segments < s: lane i
  // loads total i, one exclusive wave scan gives every prefix, and each unit
  // reads its own with a uniform readlane (NSEG <= 64), instead of every
  // lane reading all NSEG totals
  static_assert(NSEG <= 64, "segment totals are scanned across one wave");
  const int wu = __builtin_amdgcn_readfirstlane(w);
  A base[U][C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    A w0 = (A)0;
#pragma unroll
    for (int i = 0; i < NW; ++i) w0 += hsum[i * C + c];
    const A tv = lane < NSEG ? tot[lane * C + c] : (A)0;
    const A ex = wave_incl_scan(tv) - tv;
#pragma unroll
    for (int u = 0; u < U; ++u) base[u][c] = w0 + readlane(ex, u * NW + wu);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if constexpr (HS) {
      const long long sb = t0 + (long long)(u * WG + w * 64) * F;
#pragma unroll
      for (int r = 0; r < F; ++r) {
        const long long f = sb + r * 64 + lane;
        if (tile_full || f < nframes)
#pragma unroll
          for (int c = 0; c < C; ++c) out[f * C + c] = to_out<T, A, DV>(base[u][c] + v[u][r][c], p.o);
      }
      continue;
    }
    const long long f = t0 + (long long)(u * WG + tid) * F;
    U_t y;
    if constexpr (kRC) {
      const int j = u * WG + tid;
      const U_t xu = IO::load(stage + (Hu + j) * VE);
      const U_t xk = stage_xk(j);
      A run[C];
#pragma unroll
      for (int c = 0; c < C; ++c) run[c] = (A)0;
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) {
          run[c] += to_acc<A>(xu.e[fr * C + c]) - to_acc<A>(xk.e[fr * C + c]);
          y.e[fr * C + c] = to_out<T, A, DV>(base[u][c] + lx[u][c] + run[c], p.o);
        }
    } else {
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) y.e[fr * C + c] = to_out<T, A, DV>(base[u][c] + lx[u][c] + v[u][fr][c], p.o);
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
