// mavg_wide.hpp -- the wide-frame tile scan (wide_tile_kernel): the Blelloch
// flavour for multi-channel frames (fp32 C = 2, 4, 8), built around chunks of
// consecutive frames per lane.
#pragma once

#include "mavg_device.hpp"

namespace mavg {

// ----------------------------------------------------------------------------
// Why a separate kernel.  tile_scan_kernel gives each lane one 16-B unit: 4
// fp32 frames of one channel (mono), but 2 frames of 2 channels, or 1 frame of
// 4, or half a frame of 8.  Every channel a lane holds costs one 64-lane fp64
// DPP scan, so per 16 B the scan work grows with C (C=4: 4 scans per 16 B,
// 0.50 of peak; C=8 with 32-B units: 0.20).  Here every lane owns a CHUNK of
// P consecutive frames (64 B for C = 2 (P=8) and 4 (P=4), 128 B for C = 8
// (P=4)): the serial in-lane sum runs over P frames per channel, and each
// channel costs one wave scan per chunk -- at most one scan per 16 B, the mono
// kernel's rate, for every C.
//
// The chunks are read from an LDS stage that LDS-DMA fills with whole 1-KiB
// pieces (global_load_lds_dwordx4: coalesced, no staging registers).  A lane
// reading its own 64 or 128 contiguous bytes with ds_read_b128 would be a 4-
// or 8-way bank conflict on the linear layout (16 lanes of a ds_read_b128 group
// hit the same four 16-B slots of the 256-B bank row), so the stage is
// XOR-swizzled: logical granule g (16 B) lives in slot g ^ ((g >> 4) & QM),
// QM = 3 for 64-B chunks, 7 for 128-B chunks.  The swizzle only permutes the
// granules inside each aligned 128 B, so a DMA wave-instruction still reads
// 1 KiB of contiguous global memory: lane l of the piece fetches the logical
// granule its slot holds (the map is an involution).  With it every chunk
// read, of x and of x[n-k] at ANY shift (including the half-granule shift of
// odd k at C = 2), is conflict-free (enumerated against the ds_read_b128 lane
// groups of MI355X_MICROARCH.md, DESIGN.md "wide_tile_kernel").
//
// Outputs leave through LDS as well: after the block's last read of the stage,
// each wave writes its chunks' results into its own part of the tile region
// (swizzle g ^ ((g >> 3) & 7): conflict-free ds_write_b128) and reads
// them back slot-contiguous, so every global store instruction writes 1 KiB
// of contiguous output (a lane-strided 64-B/128-B store would touch 64
// different lines per instruction).
//
// The rest is the tile kernel's scheme: the k-frame halo staged in front of
// the tile gives W[t0-1] (block reduction) and every x[n-k]; the wave-segment
// totals are scanned once across a wave; XCD-remapped flat tiles; the pass-2
// prefix is rebuilt from the stage (RC) so only C lane totals per row live
// across the second barrier.
// ----------------------------------------------------------------------------
struct WideParams {
  const void* in;
  void* out;
  const void* hist;
  long long nframes;
  long long ntiles;
  int k;
  int halo_g;     // staged halo granules (16 B each): a multiple of 16 (whole 256-B rows), >= k*C elements
  int xk_off;     // (-k*C) mod EPG: element offset of x[n-k] inside its granule (uniform)
  int xcd_remap;  // remap_tile mode
  int pre;        // frames in front of `in` that are readable signal (load_elem)
  OutParams o;
};

// stage: logical granule -> LDS slot (QM = 3 for 64-B chunks, 7 for 128-B chunks)
template <int QM>
__device__ __forceinline__ int stage_slot(int g) {
  return g ^ ((g >> 4) & QM);
}
// output region of one wave: lane l's chunk granule i is logical l*G + i;
// keyed on bits 3-5, so the map is an involution and the ds_write_b128 of 8
// consecutive lanes (64-B or 128-B chunks) hit 8 distinct 16-B slots of a
// 128-B bank row
__device__ __forceinline__ int out_slot(int g) {
  return g ^ ((g >> 3) & 7);
}

// extract elements [o, o + N) of a flat register array of N + EPG elements; o
// uniform, one of the multiples of STEP below EPG (a chain of scalar compares)
template <int O, int STEP, int EPG, typename T, int N>
__device__ __forceinline__ void extract_chunk(const T (&flat)[N + EPG], T (&r)[N], int o) {
  if constexpr (O + STEP >= EPG) {
#pragma unroll
    for (int i = 0; i < N; ++i) r[i] = flat[O + i];
  } else {
    if (o == O) {
#pragma unroll
      for (int i = 0; i < N; ++i) r[i] = flat[O + i];
      return;
    }
    extract_chunk<O + STEP, STEP, EPG, T, N>(flat, r, o);
  }
}

// NT: kNtStore / kNtSplit / kNtHalo as in tile_scan_kernel (the tile's loads
//     non-temporal except the tail the next tile's halo re-reads; halo loads
//     non-temporal; non-temporal output stores).
template <typename T, typename A, int C, int P, int U, int WG, int NT, int DV = 0>
__global__ __launch_bounds__(WG) void wide_tile_kernel(WideParams p) {
  constexpr int NW = WG / 64;
  constexpr int EPG = 16 / (int)sizeof(T);  // elements per 16-B granule
  constexpr int CE = P * C;                 // elements per lane chunk
  constexpr int G = CE / EPG;               // granules per lane chunk
  static_assert(CE % EPG == 0 && (G == 4 || G == 8), "64-B or 128-B chunks");
  constexpr int QM = G == 4 ? 3 : 7;
  constexpr int TF = WG * P * U;  // tile frames
  constexpr int TG = WG * U * G;  // tile granules
  constexpr int NSEG = U * NW;
  using IO = UnitIO<T, EPG>;
  using Gr = Unit<T, EPG>;

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int Hg = p.halo_g;
  unsigned char* sb = smem;                                    // [Hg + TG] swizzled granules
  A* tot = reinterpret_cast<A*>(smem + (Hg + TG) * 16);        // [NSEG][C] segment totals
  A* hsum = tot + NSEG * C;                                    // [NW][C] halo partial sums
  auto gread = [&](int g) -> Gr { return IO::load(reinterpret_cast<const T*>(sb + stage_slot<QM>(g) * 16)); };

  const T* __restrict__ in = static_cast<const T*>(p.in);
  T* __restrict__ out = static_cast<T*>(p.out);
  const T* __restrict__ hist = static_cast<const T*>(p.hist);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int wq = __builtin_amdgcn_readfirstlane(w);
  const int k = p.k;
  const long long nframes = p.nframes;

  const long long tile = remap_tile(blockIdx.x, gridDim.x, p.xcd_remap);
  const long long t0 = tile * TF;
  const int Hf = Hg * EPG / C;  // staged halo frames (>= k)
  const long long h0 = t0 - Hf;
  MAVG_DCHECK(tile >= 0 && tile < p.ntiles && t0 < nframes, "wide tile index", tile, p.ntiles);
  MAVG_DCHECK(Hf >= k && Hg % 16 == 0, "wide halo", Hf, k);
  const bool tile_full = t0 + TF <= nframes;
  const bool dma = tile_full && h0 >= 0;  // uniform

  // ---- stage: halo + tile, swizzled ----
  if (dma) {
    const T* src0 = in + h0 * C;  // logical granule 0
#pragma unroll
    for (int i = 0; i < U * G; ++i) {
      const int gl = stage_slot<QM>(Hg + i * WG + tid);  // the logical granule this lane's slot holds
      unsigned char* d = sb + (Hg + i * WG + wq * 64) * 16;
      if constexpr ((NT & kNtSplit) != 0) {
        // the last Hg granules of the tile are the next tile's halo: default policy (L2)
        if (gl >= TG) glds16<false>(src0 + (long long)gl * EPG, d);
        else glds16<true>(src0 + (long long)gl * EPG, d);
      } else {
        glds16<(NT & kNtLoad) != 0>(src0 + (long long)gl * EPG, d);
      }
    }
    for (int j0 = 0; j0 < Hg; j0 += WG) {
      const int s = j0 + tid;
      if (s < Hg) glds16<(NT & kNtHalo) != 0>(src0 + (long long)stage_slot<QM>(s) * EPG, sb + (j0 + wq * 64) * 16);
    }
  } else {
    // edge tiles (the first tiles, the ragged last one): element loads through
    // load_elem (history, the peeled head, zeros), stored to the swizzled slots
#pragma unroll 1
    for (int gl = tid; gl < Hg + TG; gl += WG) {
      Gr u;
#pragma unroll
      for (int i = 0; i < EPG; ++i) {
        const int e = gl * EPG + i;
        u.e[i] = load_elem(in, hist, h0 + e / C, e % C, C, nframes, k, p.pre);
      }
      IO::store(reinterpret_cast<T*>(sb + stage_slot<QM>(gl) * 16), u);
    }
  }
  __syncthreads();

  // ---- halo reduction: W[t0-1] = the k frames before t0 = stage elements [(Hf-k)C, Hf C) ----
  {
    const int e0 = (Hf - k) * C;
    const int g0 = e0 / EPG;
    A hs[EPG];
#pragma unroll
    for (int i = 0; i < EPG; ++i) hs[i] = (A)0;
    for (int gl = g0 + tid; gl < Hg; gl += WG) {
      const Gr u = gread(gl);
#pragma unroll
      for (int i = 0; i < EPG; ++i)
        if (gl * EPG + i >= e0) hs[i] += to_acc<A>(u.e[i]);
    }
    // element i of this thread's granules is channel (cb + i) mod C (its
    // granules are WG apart: WG*EPG elements, whole frames)
    const int cb = C <= EPG ? 0 : ((g0 + tid) * EPG) % C;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      A part = (A)0;
#pragma unroll
      for (int i = 0; i < EPG; ++i) {
        if constexpr (C <= EPG) {
          if (i % C == c) part += hs[i];
        } else {
          if (cb + i == c) part += hs[i];
        }
      }
      const A r = readlane(wave_incl_scan(part), 63);
      if (lane == 0) hsum[w * C + c] = r;
    }
  }

  // chunk j: x from the stage, and x[n-k] (an element shift of the same stage)
  auto x_chunk = [&](int j, T (&xv)[CE]) {
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const Gr g = gread(Hg + j * G + i);
#pragma unroll
      for (int e = 0; e < EPG; ++e) xv[i * EPG + e] = g.e[e];
    }
  };
  auto xk_chunk = [&](int j, T (&xk)[CE]) {
    const int e = Hg * EPG + j * CE - k * C;  // stage element of x[n-k] for the chunk's first frame
    MAVG_DCHECK(e >= 0 && e + CE <= (Hg + TG) * EPG, "wide x[n-k] stage index", e, j);
    if constexpr (C % EPG == 0) {
#pragma unroll
      for (int i = 0; i < G; ++i) {
        const Gr g = gread(e / EPG + i);
#pragma unroll
        for (int q = 0; q < EPG; ++q) xk[i * EPG + q] = g.e[q];
      }
    } else {
      if (p.xk_off == 0) {
#pragma unroll
        for (int i = 0; i < G; ++i) {
          const Gr g = gread(e / EPG + i);
#pragma unroll
          for (int q = 0; q < EPG; ++q) xk[i * EPG + q] = g.e[q];
        }
      } else {
        const int gs = (e - p.xk_off) / EPG;
        T flat[CE + EPG];
#pragma unroll
        for (int i = 0; i <= G; ++i) {
          const Gr g = gread(gs + i);
#pragma unroll
          for (int q = 0; q < EPG; ++q) flat[i * EPG + q] = g.e[q];
        }
        extract_chunk<C, C, EPG, T, CE>(flat, xk, p.xk_off);
      }
    }
  };

  // ---- pass 1: chunk totals, wave scans, segment totals ----
  A lx[U][C];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int j = u * WG + tid;
    T xv[CE], xk[CE];
    x_chunk(j, xv);
    xk_chunk(j, xk);
    A run[C];
#pragma unroll
    for (int c = 0; c < C; ++c) run[c] = (A)0;
#pragma unroll
    for (int fr = 0; fr < P; ++fr)
#pragma unroll
      for (int c = 0; c < C; ++c) run[c] += to_acc<A>(xv[fr * C + c]) - to_acc<A>(xk[fr * C + c]);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const A incl = wave_incl_scan(run[c]);
      lx[u][c] = incl - run[c];
      const A segtot = readlane(incl, 63);
      if (lane == 0) tot[(u * NW + w) * C + c] = segtot;
    }
  }
  __syncthreads();

  // ---- carry: halo sum + earlier segments (one wave scan of the segment totals) ----
  static_assert(NSEG <= 64, "segment totals are scanned across one wave");
  A base[U][C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    A w0 = (A)0;
#pragma unroll
    for (int i = 0; i < NW; ++i) w0 += hsum[i * C + c];
    const A tv = lane < NSEG ? tot[lane * C + c] : (A)0;
    const A ex = wave_incl_scan(tv) - tv;
#pragma unroll
    for (int u = 0; u < U; ++u) base[u][c] = w0 + readlane(ex, u * NW + wq) + lx[u][c];
  }

  // ---- pass 2: the in-chunk prefixes rebuilt from the stage, outputs ----
  T yv[U][CE];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int j = u * WG + tid;
    T xv[CE], xk[CE];
    x_chunk(j, xv);
    xk_chunk(j, xk);
    A run[C];
#pragma unroll
    for (int c = 0; c < C; ++c) run[c] = base[u][c];
#pragma unroll
    for (int fr = 0; fr < P; ++fr)
#pragma unroll
      for (int c = 0; c < C; ++c) {
        run[c] += to_acc<A>(xv[fr * C + c]) - to_acc<A>(xk[fr * C + c]);
        yv[u][fr * C + c] = to_out<T, A, DV>(run[c], p.o);
      }
  }

  if (!tile_full) {  // the ragged last tile: element stores
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long f = t0 + (long long)(u * WG + tid) * P;
#pragma unroll
      for (int fr = 0; fr < P; ++fr)
        if (f + fr < nframes)
#pragma unroll
          for (int c = 0; c < C; ++c) out[(f + fr) * C + c] = yv[u][fr * C + c];
    }
    return;
  }
  // ---- outputs through LDS: 1 KiB of contiguous output per store instruction ----
  __syncthreads();  // every read of the stage is done; the tile region takes the outputs
#pragma unroll
  for (int u = 0; u < U; ++u) {
    unsigned char* rb = sb + (Hg + (u * WG + wq * 64) * G) * 16;  // this wave's region (64 chunks)
#pragma unroll
    for (int i = 0; i < G; ++i) {
      Gr g;
#pragma unroll
      for (int e = 0; e < EPG; ++e) g.e[e] = yv[u][i * EPG + e];
      IO::store(reinterpret_cast<T*>(rb + out_slot(lane * G + i) * 16), g);
    }
  }
  // the wave reads back only its own region: wave-level ordering suffices
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const unsigned char* rb = sb + (Hg + (u * WG + wq * 64) * G) * 16;
    T* ob = out + (t0 + (long long)(u * WG + wq * 64) * P) * C;  // the wave's 64 chunks, contiguous
#pragma unroll
    for (int r = 0; r < G; ++r) {
      const int s = r * 64 + lane;
      const Gr g = IO::load(reinterpret_cast<const T*>(rb + s * 16));
      IO::template store<(NT & kNtStore) != 0>(ob + out_slot(s) * EPG, g);
    }
  }
}

}  // namespace mavg
