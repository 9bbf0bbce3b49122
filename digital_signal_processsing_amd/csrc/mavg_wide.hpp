// mavg_wide.hpp -- the wide-frame tile scan (wide_tile_kernel): the Blelloch
// flavour for multi-channel frames (fp32 C = 2, 4, 8), built around chunks of
// consecutive frames per lane.
#pragma once

#include <type_traits>

#include "mavg_device.hpp"
#include "mavg_lookback.hpp"

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

// the chunk's registers are raw dwords (a 16-B granule = 4 dwords): element
// i of a chunk of T
template <typename T>
__device__ __forceinline__ T chunk_elem(const uint32_t* w, int i) {
  if constexpr (sizeof(T) == 4) {
    return __uint_as_float(w[i]);
  } else {
    return (T)(int16_t)(uint16_t)(w[i >> 1] >> (16 * (i & 1)));
  }
}
// r[i] = flat[o + i] for a uniform dword offset o, one of the multiples of
// STEP below 4 (a chain of scalar compares, one static copy taken)
template <int O, int STEP, int N>
__device__ __forceinline__ void shift_words(const uint32_t (&flat)[N + 4], uint32_t (&r)[N], int o) {
  if constexpr (O + STEP >= 4) {
#pragma unroll
    for (int i = 0; i < N; ++i) r[i] = flat[O + i];
  } else {
    if (o == O) {
#pragma unroll
      for (int i = 0; i < N; ++i) r[i] = flat[O + i];
      return;
    }
    shift_words<O + STEP, STEP, N>(flat, r, o);
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
  static_assert((C * sizeof(T)) % 4 == 0, "frames of whole dwords: x[n-k] shifts by whole dwords");
  constexpr int NWD = G * 4;  // dwords per chunk
  auto gwords = [&](int g, uint32_t* d) {
    const u32x4 v = *reinterpret_cast<const u32x4*>(sb + stage_slot<QM>(g) * 16);
    d[0] = v[0];
    d[1] = v[1];
    d[2] = v[2];
    d[3] = v[3];
  };
  auto x_chunk = [&](int j, uint32_t (&xv)[NWD]) {
#pragma unroll
    for (int i = 0; i < G; ++i) gwords(Hg + j * G + i, xv + 4 * i);
  };
  auto xk_chunk = [&](int j, uint32_t (&xk)[NWD]) {
    const int e = Hg * EPG + j * CE - k * C;  // stage element of x[n-k] for the chunk's first frame
    MAVG_DCHECK(e >= 0 && e + CE <= (Hg + TG) * EPG, "wide x[n-k] stage index", e, j);
    constexpr int kStep = C * (int)sizeof(T) / 4;  // dwords per frame
    if constexpr (kStep % 4 == 0) {
#pragma unroll
      for (int i = 0; i < G; ++i) gwords(e / EPG + i, xk + 4 * i);
    } else {
      if (p.xk_off == 0) {
#pragma unroll
        for (int i = 0; i < G; ++i) gwords(e / EPG + i, xk + 4 * i);
      } else {
        const int gs = (e - p.xk_off) / EPG;
        uint32_t flat[NWD + 4];
#pragma unroll
        for (int i = 0; i <= G; ++i) gwords(gs + i, flat + 4 * i);
        shift_words<kStep, kStep, NWD>(flat, xk, p.xk_off * (int)sizeof(T) / 4);
      }
    }
  };
  auto d_at = [&](const uint32_t (&xv)[NWD], const uint32_t (&xk)[NWD], int i) -> A {
    return to_acc<A>(chunk_elem<T>(xv, i)) - to_acc<A>(chunk_elem<T>(xk, i));
  };

  // ---- pass 1: chunk totals, wave scans, segment totals ----
  A lx[U][C];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int j = u * WG + tid;
    uint32_t xv[NWD], xk[NWD];
    x_chunk(j, xv);
    xk_chunk(j, xk);
    A run[C];
#pragma unroll
    for (int c = 0; c < C; ++c) run[c] = (A)0;
#pragma unroll
    for (int fr = 0; fr < P; ++fr)
#pragma unroll
      for (int c = 0; c < C; ++c) run[c] += d_at(xv, xk, fr * C + c);
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
    uint32_t xv[NWD], xk[NWD];
    x_chunk(j, xv);
    xk_chunk(j, xk);
    A run[C];
#pragma unroll
    for (int c = 0; c < C; ++c) run[c] = base[u][c];
#pragma unroll
    for (int fr = 0; fr < P; ++fr)
#pragma unroll
      for (int c = 0; c < C; ++c) {
        run[c] += d_at(xv, xk, fr * C + c);
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

// ----------------------------------------------------------------------------
// chan_tile_kernel: the wide tile with lanes that own ONE channel each (round
// 4, fp32 C = 8 and 4).  In wide_tile_kernel a lane's chunk holds every
// channel of its P frames, so each chunk costs C fp64 wave scans (C = 8: eight
// 6-step scans per 128 B).  Here lane = b * C + c owns channel c of Q
// consecutive frames (frame block b of NB = 64 / C per wave): its in-lane sum
// runs over Q frames of one channel, and ONE scan across the NB lanes of its
// channel (log2 NB ds_bpermute steps at stride C, 2C, .. lanes) serves all C
// channels at once.
//
// The stage is the wide tile's (halo + tile by LDS-DMA, 16-B granules) with a
// swizzle for the lane-per-channel reads: ds_read_b32 of element (frame
// m + b*Q, channel c) for the 64 lanes hits granules m*GPF + b*Q*GPF + c/4 --
// the same 16-B slot of the bank row for every b on the linear layout (an NB-
// way conflict).  Slot(g) = g ^ (((g >> SH) & (NB - 1)) << LG), SH =
// log2(Q * GPF), LG = log2(GPF) (GPF granules per frame): the key is b plus a
// constant for every lane of one read (any m: the low SH bits of m * GPF + c/4
// never carry into bit SH), so the NB blocks land in NB distinct bank groups,
// the c/4 bits in the rest: 64 distinct banks.  Like the wide tile's swizzle it
// permutes granules inside aligned 256 B (an involution), so every LDS-DMA
// instruction still reads 1 KiB of contiguous global memory, and the outputs
// written back in the same layout leave as 1-KiB contiguous stores.
// ----------------------------------------------------------------------------
constexpr int ilog2c(int v) { return v <= 1 ? 0 : 1 + ilog2c(v / 2); }

template <int C, int Q>
__device__ __forceinline__ int chan_slot(int g) {
  constexpr int NB = 64 / C, GPF = C / 4;
  constexpr int SH = ilog2c(Q * GPF), LG = ilog2c(GPF);
  return g ^ (((g >> SH) & (NB - 1)) << LG);
}

// XG (windows of at least a tile, k >= TF): only the halo is staged; each lane
// loads its own Q values of x straight from global memory (4-B loads, 8
// 32-B segments per wave instruction, every line used whole over 4 frames),
// since every x[n-k] of the tile then lies in the halo.  Half the LDS at
// k = TF (C = 8, k = 1024: 32 KiB, four workgroups per CU instead of two);
// the outputs are staged in the halo region after the last read of it.
//
// int16 (round 5, C = 8): a lane owns one DWORD COLUMN of the frame -- two
// adjacent channels -- so the addressing is exactly fp32 C = 4's (16-B frames,
// CL = 4 columns, NB = 16 blocks per wave, conflict-free ds_read_b32 of the
// chan_slot stage), with E = 2 int32 accumulators per lane; one ds_read_b32
// serves two samples, half the LDS instructions of a lane per channel.
template <typename T> struct ChanElem;  // a dword of the stage as E samples
template <> struct ChanElem<float> {
  static constexpr int E = 1;
  static __device__ __forceinline__ float get(uint32_t w, int) { return __uint_as_float(w); }
  static __device__ __forceinline__ uint32_t put(const float (&y)[1]) { return __float_as_uint(y[0]); }
};
template <> struct ChanElem<int16_t> {
  static constexpr int E = 2;
  static __device__ __forceinline__ int16_t get(uint32_t w, int e) { return (int16_t)(uint16_t)(w >> (16 * e)); }
  static __device__ __forceinline__ uint32_t put(const int16_t (&y)[2]) {
    return (uint32_t)(uint16_t)y[0] | ((uint32_t)(uint16_t)y[1] << 16);
  }
};

// XL (round 6, the halo-only forms): a lane's column of P frames j0 .. j0 + P - 1 loaded as
// 16-B pieces of whole frames and turned into the column by quad transposes (quad_transpose4),
// once the first barrier has passed so the loads stay in flight behind everything issued after
// them.  Lane l = cl of its block's CL lanes loads, for each group of 4 frames j0 + 4m .. + 3,
// the 16 bytes at frame j0 + 4m + (cl mod 4), byte 16 (cl / 4) -- the block's CL lanes read the
// group's 4 CL dwords, 64 (CL = 4) or 128 (CL = 8) contiguous bytes per wave instruction.  In
// bit terms the lane index is (byte half, frame bits 1..0) and the 4 registers are dword bits
// 1..0; the transpose swaps lane bits 1..0 with register bits 1..0, leaving dword cl of the 4
// frames in the lane's 4 registers.  The 4-B column loads fetched 16 (CL = 4) or 8 (CL = 8)
// separate 16-B / 32-B pieces per wave instruction: four times the vector-memory transactions
// for the same bytes.  Every tile loads this way: its frames are >= 0, so only the end needs
// care -- frames past it read the last frame (outputs there are not stored).  No branch between
// two load forms: such a merge made the compiler wait for these loads before issuing the stage.
template <int P, int CL>
__device__ __forceinline__ void xl_load(const void* in, long long f0, int cl, long long nframes, uint32_t (&xr)[P]) {
  static_assert(P % 4 == 0 && (CL == 4 || CL == 8), "whole quads of frames, 16- or 32-B frames");
  const uint32_t* in32 = static_cast<const uint32_t*>(in);
  const long long last = nframes - 1;
#pragma unroll
  for (int m = 0; m < P / 4; ++m) {
    const long long f = f0 + 4 * m + (cl & 3);
    const u32x4 v = *reinterpret_cast<const u32x4*>(in32 + (f < last ? f : last) * CL + 4 * (cl >> 2));
#pragma unroll
    for (int q = 0; q < 4; ++q) xr[4 * m + q] = v[q];
  }
}
template <int P>
__device__ __forceinline__ void xl_transpose(uint32_t (&xr)[P], int cl) {
#pragma unroll
  for (int m = 0; m < P / 4; ++m) {
    uint32_t q4[4] = {xr[4 * m], xr[4 * m + 1], xr[4 * m + 2], xr[4 * m + 3]};
    quad_transpose4(q4, cl & 3);
#pragma unroll
    for (int f = 0; f < 4; ++f) xr[4 * m + f] = q4[f];
  }
}

// IP (XG only, the launcher's choice when the staged halo is exactly k frames): each output is
// written in pass 2 over the x[n-k] it last read -- the same lane and address, as in the wide
// look-ahead -- so no barrier before the output stage and no Q output registers
template <typename T, typename A, int C, int Q, int WG, int NT, int DV = 0, bool XG = false, bool IP = false,
          int XL = 0>
__global__ __launch_bounds__(WG) void chan_tile_kernel(WideParams p) {
  static_assert(!IP || XG, "in-place outputs need the halo-only stage");
  using CE = ChanElem<T>;
  constexpr int E = CE::E;      // samples (channels) per dword
  constexpr int CL = C / E;     // dword columns per frame
  static_assert(C % E == 0 && (CL == 4 || CL == 8), "frames of 16 or 32 bytes");
  static_assert(XL == 0 || XG, "16-B frame-piece loads: the halo-only form");
  constexpr int NW = WG / 64;
  constexpr int NB = 64 / CL;   // frame blocks per wave
  constexpr int GPF = CL / 4;   // 16-B granules per frame
  constexpr int EPG = 16 / (int)sizeof(T);  // samples per granule
  static_assert(ilog2c(GPF) + ilog2c(NB) == 4 && Q * GPF >= 16, "the key spans one bank row, outside its bits");
  constexpr int WF = NB * Q;    // frames per wave
  constexpr int TF = NW * WF;   // tile frames
  constexpr int TG = TF * GPF;  // tile granules
  using IO = UnitIO<T, EPG>;
  using Gr = Unit<T, EPG>;

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int Hg = p.halo_g;
  unsigned char* sb = smem;                              // [Hg + TG] swizzled granules
  A* tot = reinterpret_cast<A*>(smem + (Hg + (XG ? 0 : TG)) * 16);  // [NW][C] wave-segment totals
  A* hsum = tot + NW * C;                                // [NW][C] halo partial sums
  const uint32_t* sw32 = reinterpret_cast<const uint32_t*>(sb);
  // stage dword d (frame * CL + column), swizzled
  auto dword_at = [&](int d) -> uint32_t { return sw32[chan_slot<CL, Q>(d >> 2) * 4 + (d & 3)]; };

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
  MAVG_DCHECK(tile >= 0 && tile < p.ntiles && t0 < nframes, "chan tile index", tile, p.ntiles);
  MAVG_DCHECK(Hf >= k && Hg % 16 == 0, "chan halo", Hf, k);
  MAVG_DCHECK(!XG || (k >= TF && Hg >= TG), "chan XG window", k, TF);
  const bool tile_full = t0 + TF <= nframes;
  constexpr int kTileStaged = XG ? 0 : TG;  // granules of the tile in the stage
  const int c = lane & (CL - 1);  // the lane's dword column: channels c*E .. c*E + E - 1
  const int b = lane / CL;
  const int jl = w * WF + b * Q;  // tile frame of the lane's first frame
  uint32_t xr[XG ? Q : 1];
  if constexpr (XG && XL == 1) {
    xl_load<Q, CL>(in, t0 + jl, c, nframes, xr);
  } else if constexpr (XG) {  // the lane's x, issued before the stage
    if (tile_full) {
      const uint32_t* in32 = reinterpret_cast<const uint32_t*>(in);
#pragma unroll
      for (int i = 0; i < Q; ++i) xr[i] = in32[(t0 + jl + i) * CL + c];
    } else {
#pragma unroll
      for (int i = 0; i < Q; ++i) {
        T v[E];
#pragma unroll
        for (int e = 0; e < E; ++e) v[e] = load_elem(in, hist, t0 + jl + i, c * E + e, C, nframes, k, p.pre);
        xr[i] = CE::put(v);
      }
    }
  }

  // ---- stage: halo + tile, swizzled ----
  if (tile_full && h0 >= 0) {
    const T* src0 = in + h0 * C;  // logical granule 0
#pragma unroll
    for (int i = 0; i < kTileStaged / WG; ++i) {
      const int gl = chan_slot<CL, Q>(Hg + i * WG + tid);  // the logical granule this lane's slot holds
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
      if (s < Hg) glds16<(NT & kNtHalo) != 0>(src0 + (long long)chan_slot<CL, Q>(s) * EPG, sb + (j0 + wq * 64) * 16);
    }
  } else {
    // edge tiles: element loads through load_elem (history, peeled head, zeros)
#pragma unroll 1
    for (int gl = tid; gl < Hg + kTileStaged; gl += WG) {
      Gr u;
#pragma unroll
      for (int i = 0; i < EPG; ++i) {
        const int e = gl * EPG + i;
        u.e[i] = load_elem(in, hist, h0 + e / C, e % C, C, nframes, k, p.pre);
      }
      IO::store(reinterpret_cast<T*>(sb + chan_slot<CL, Q>(gl) * 16), u);
    }
  }
  __syncthreads();

  // ---- halo reduction: W[t0-1] = stage elements [(Hf-k)C, Hf C), per channel ----
  {
    const int e0 = (Hf - k) * C;
    const int g0 = e0 / EPG;
    A hs[EPG];
#pragma unroll
    for (int i = 0; i < EPG; ++i) hs[i] = (A)0;
    for (int gl = g0 + tid; gl < Hg; gl += WG) {
      const Gr u = IO::load(reinterpret_cast<const T*>(sb + chan_slot<CL, Q>(gl) * 16));
#pragma unroll
      for (int i = 0; i < EPG; ++i)
        if (gl * EPG + i >= e0) hs[i] += to_acc<A>(u.e[i]);
    }
    // element i of this thread's granules is channel (cb + i) mod C (granules WG apart: whole frames)
    const int cb = ((g0 + tid) * EPG) % C;
    if constexpr (EPG < C && C % EPG == 0) {
      // fp32 C = 8: cb repeats every C / EPG lanes (the lane's parity), and those lanes' elements
      // are the C channels once each -- butterflies over the lanes of one residue instead of C
      // whole-wave fp64 scans (in-process, profiles/r05_tuning/wide/cand_chanbf_*: k=1536 0.649 ->
      // 0.663, k=1024 0.738 -> 0.740)
#pragma unroll
      for (int sh = C / EPG; sh < 64; sh <<= 1)
#pragma unroll
        for (int i = 0; i < EPG; ++i) hs[i] += __shfl_xor(hs[i], sh, 64);
      if (lane < C / EPG)
#pragma unroll
        for (int i = 0; i < EPG; ++i) hsum[w * C + (cb + i) % C] = hs[i];
    } else {
#pragma unroll
      for (int ch = 0; ch < C; ++ch) {
        A part = (A)0;
#pragma unroll
        for (int i = 0; i < EPG; ++i)
          if ((cb + i) % C == ch) part += hs[i];
        const A r = readlane(wave_incl_scan(part), 63);
        if (lane == 0) hsum[w * C + ch] = r;
      }
    }
  }

  // ---- pass 1: the lane's channels over its Q frames; the scan across its NB lanes ----
  if constexpr (XL == 1) xl_transpose<Q>(xr, c);
  const int f0 = Hf + jl;  // stage frame of the lane's first frame
  auto xv = [&](int i) -> uint32_t {
    if constexpr (XG) return xr[i];
    else return dword_at((f0 + i) * CL + c);
  };
  A run[E];
#pragma unroll
  for (int e = 0; e < E; ++e) run[e] = (A)0;
#pragma unroll
  for (int i = 0; i < Q; ++i) {
    const uint32_t x = xv(i), xk = dword_at((f0 + i - k) * CL + c);
#pragma unroll
    for (int e = 0; e < E; ++e) run[e] += to_acc<A>(CE::get(x, e)) - to_acc<A>(CE::get(xk, e));
  }
  // Kogge-Stone over the NB blocks: steps of 1, 2, 4 .. blocks = CL, 2CL, 4CL ..
  // lanes.  Every step crosses 16-lane rows for half the lanes (block b - 1 of
  // an even block lies in the previous row), so row_shr DPP cannot serve it:
  // ds_bpermute (shfl_up), every lane taking part
  A incl[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    incl[e] = run[e];
#pragma unroll
    for (int s = CL; s < 64; s <<= 1) {
      A t = shfl_up(incl[e], s);
      t = lane >= s ? t : (A)0;
      incl[e] += t;
    }
    if (b == NB - 1) tot[w * C + c * E + e] = incl[e];  // the wave segment's total of the channel
  }
  __syncthreads();

  // ---- carry: halo sum + the earlier waves' segments of this channel, in wave order ----
  A base[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int ch = c * E + e;
    base[e] = (A)0;
#pragma unroll
    for (int i = 0; i < NW; ++i) base[e] += hsum[i * C + ch];
#pragma unroll
    for (int i = 0; i < NW - 1; ++i)
      if (i < wq) base[e] += tot[i * C + ch];
    base[e] += incl[e] - run[e];
  }

  // ---- pass 2: the prefix rebuilt from the stage, outputs ----
  uint32_t* sww = reinterpret_cast<uint32_t*>(sb);
  // the outputs in registers, then the ragged tile's element stores or the LDS output stage
  auto pass2_regs = [&]() -> bool {
    uint32_t yv[Q];
#pragma unroll
    for (int i = 0; i < Q; ++i) {
      const uint32_t x = xv(i), xk = dword_at((f0 + i - k) * CL + c);
      T y[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        base[e] += to_acc<A>(CE::get(x, e)) - to_acc<A>(CE::get(xk, e));
        y[e] = to_out<T, A, DV>(base[e], p.o);
      }
      yv[i] = CE::put(y);
    }
    if (!tile_full) {  // the ragged last tile: element stores
      const long long f = t0 + (long long)jl;
#pragma unroll
      for (int i = 0; i < Q; ++i)
        if (f + i < nframes)
#pragma unroll
          for (int e = 0; e < E; ++e) out[(f + i) * C + c * E + e] = CE::get(yv[i], e);
      return false;
    }
    // ---- outputs through LDS (the stage layout), 1 KiB of contiguous output per store ----
    __syncthreads();  // every read of the stage is done
    const int fo = (XG ? 0 : Hf) + jl;  // XG: the outputs take the halo region (Hg >= TG granules)
#pragma unroll
    for (int i = 0; i < Q; ++i) {
      const int d = (fo + i) * CL + c;
      sww[chan_slot<CL, Q>(d >> 2) * 4 + (d & 3)] = yv[i];
    }
    return true;
  };
  if constexpr (IP) {
    MAVG_DCHECK(Hf == k, "in-place chan tile: halo of exactly k frames", Hf, k);
    if (!tile_full) {
      pass2_regs();
      return;
    }
    // the slot addresses from a value the compiler cannot prove equal to pass 1's (it would keep
    // pass 1's Q addresses live across the carry), as in the wide look-ahead
    int jx = jl;
    asm volatile("" : "+v"(jx));
#pragma unroll
    for (int i = 0; i < Q; ++i) {
      // groups of 8 frames the scheduler may not mix (the wide look-ahead's pass 2): bounded live
      // LDS reads and fp64 conversions
      if (i % 8 == 0 && i > 0) __builtin_amdgcn_sched_barrier(0);
      const int d = (jx + i) * CL + c;  // = (f0 + i - k) CL + c: this lane's x[n-k], its output slot
      uint32_t* sl = sww + chan_slot<CL, Q>(d >> 2) * 4 + (d & 3);
      const uint32_t x = xv(i), xk = *sl;
      T y[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        base[e] += to_acc<A>(CE::get(x, e)) - to_acc<A>(CE::get(xk, e));
        y[e] = to_out<T, A, DV>(base[e], p.o);
      }
      *sl = CE::put(y);
    }
  } else {
    if (!pass2_regs()) return;
  }
  // the wave reads back only its own frames: wave-level ordering suffices
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  constexpr int WGR = WF * GPF;  // the wave's granules
  const int rg = (XG ? 0 : Hg) + wq * WGR;
  T* ob = out + (t0 + (long long)wq * WF) * C;
#pragma unroll
  for (int r = 0; r < WGR / 64; ++r) {
    const int s = rg + r * 64 + lane;  // slot
    const Gr g = IO::load(reinterpret_cast<const T*>(sb + s * 16));
    IO::template store<(NT & kNtStore) != 0>(ob + (long long)(chan_slot<CL, Q>(s) - rg) * EPG, g);
  }
}

}  // namespace mavg

namespace mavg {

// ----------------------------------------------------------------------------
// wide_ahead_kernel: the look-ahead scan (mavg_lookback.hpp) with the wide
// in-tile scan, for multi-channel windows too long for the wide tile's
// LDS-staged halo.  The record carry is the look-ahead scan's per-tile form,
// unchanged and in its own unit layout (F frames per unit, U units per lane:
// phase A of tile t + D, the own records of the first D slots, head duty,
// bounded polling and the consumer's recompute -- the same bits whoever
// computes a record); only the in-tile scan and the outputs change:
//   - the tile itself and the shifted tile (its x[n-k]) reach two swizzled
//     LDS stages by LDS-DMA (no tile registers);
//   - lanes own chunks of P consecutive frames (mavg_wide.hpp), one wave scan
//     per channel per chunk;
//   - outputs leave through LDS as 1-KiB contiguous stores.
// Per-wave records, run totals, self-publication and the Hillis-Steele form
// stay in ahead_scan_kernel (mono / int16 paths).
// ----------------------------------------------------------------------------
// CH (round 4, fp32 C = 8): the in-tile scan of chan_tile_kernel instead of
// the chunks -- lane = b * C + c owns channel c of P (= Q) consecutive frames,
// one ds_bpermute scan across a channel's lanes, the chan_slot stage layout
// (UW = 1); the record carry is unchanged.
// XG (round 5, with CH): the tile is not staged -- each lane loads its P values
// of x straight from global memory (chan_tile_kernel's halo-only form), only
// the shifted tile is in LDS, and the outputs leave through it after its last
// read: half the LDS per workgroup (C = 8, 1024-frame tiles: 33 KiB instead of
// 65 KiB, four workgroups per CU instead of two).
// MW: the minimum waves per SIMD the register allocation must allow (0: no
// bound).  A tuning parameter only: every dispatch in the library passes 0
// (tools/tune/wide_ab.hip's `mw` variants A/B it).  The bound was measured when
// the halo-only form held 142-228 VGPRs (forcing 128 for fp32 C = 4 spilled,
// 0.612 -> 0.50 of peak); the register work that followed (126 VGPRs at C = 8,
// 92 at C = 4) reaches the LDS-sized 4 workgroups per CU without it.
// XL (round 6, XG): x as 16-B frame-piece loads plus quad transposes (xl_load), transposed after
// the first barrier so the loads stay in flight behind the stage and phase A.
template <typename T, typename A, int C, int P, int UW, int WG, int NT, int DV, int F, int U, bool CH = false,
          bool XG = false, int MW = 0, int XL = 0>
__global__ __launch_bounds__(WG, MW > 0 ? MW : 1) void wide_ahead_kernel(AheadParams p) {
  constexpr int NW = WG / 64;
  constexpr int EPG = 16 / (int)sizeof(T);
  constexpr int CE = CH ? 4 * C : P * C;   // (CH: unused)
  constexpr int G = CE / EPG;
  static_assert(CE % EPG == 0 && (G == 4 || G == 8), "64-B or 128-B chunks");
  // XG: the halo-only form, CH only (the chunk form with x chunks from global memory and outputs
  // through the shifted stage measured a tie, round 5: fp32 stereo k=44100 0.639 -> 0.645, int16 4
  // channels 0.615 -> 0.613; profiles/r05_tuning/wide/chunkxg_*)
  static_assert(!XG || CH, "the halo-only form is the channel-per-lane form's");
  using CEl = ChanElem<T>;                 // CH: a stage dword as E samples (fp32 1, int16 2)
  constexpr int E = CEl::E;
  constexpr int CL = C / E > 0 ? C / E : 1;  // CH: dword columns per frame (a lane owns one)
  static_assert(!CH || (UW == 1 && C % E == 0 && (CL == 4 || CL == 8)), "channel-per-lane form: 16- or 32-B frames");
  static_assert(XL == 0 || (XG && P % 4 == 0), "16-B frame-piece loads: the halo-only form");
  constexpr int QM = G == 4 ? 3 : 7;
  constexpr int NB = 64 / CL;              // CH: frame blocks per wave
  constexpr int WF = NB * P;               // CH: frames per wave
  constexpr int TF = CH ? NW * WF : WG * P * UW;
  static_assert(TF == WG * F * U, "the record units tile the same frames as the chunks");
  constexpr int TG = TF * C / EPG;  // tile granules
  constexpr int SG = TG + 1;       // shifted-tile granules (one more for an x[n-k] extraction)
  constexpr int NSEG = UW * NW;
  constexpr int VE = F * C;
  using IO = UnitIO<T, VE>;
  using GIO = UnitIO<T, EPG>;
  using Gr = Unit<T, EPG>;
  using SA = typename ScanAcc<T, A>::type;
  constexpr int NG = GranCount<SA>::n;

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* sstage = smem;              // [SG] shifted tile, swizzled granules (XG: then the outputs)
  unsigned char* tstage = smem + SG * 16;    // [TG] the tile, swizzled granules (then the outputs); XG: absent
  A* hsum = reinterpret_cast<A*>(tstage + (XG ? 0 : TG) * 16);  // [NW][C]
  SA* tot = reinterpret_cast<SA*>(hsum + NW * C);    // [NSEG][C]
  SA* shares = tot + NSEG * C;                         // [3][NW][C]

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

  auto map_tile = [&](unsigned b) -> long long { return remap_tile(b, gridDim.x, p.xcd_remap); };
  const long long tile = map_tile(blockIdx.x);
  const long long t0 = tile * TF;
  const int Ha = p.halo_units * F;  // the shifted stage starts Ha >= k frames before the tile
  const long long h0 = t0 - Ha;
  MAVG_DCHECK(tile >= 0 && tile < (long long)gridDim.x && t0 < nframes, "wide ahead tile index", tile, gridDim.x);
  const bool tile_full = t0 + TF <= nframes;
  const long long a = t0 - k;
  const long long jlo = a >= 0 ? (a + TF - 1) / TF : 0;
  const long long qlo = jlo, qhi = tile;  // per-tile records of the whole tiles [jlo, tile)
  // MAVG_AHEAD_TRACE (tuning builds, tools/tune/ahead_trace.py): thread 0's phase stamps, the
  // mono look-ahead's slots: 0 start, 1 phase A summed, 2 first barrier, 3 in-tile scan, 4 wave
  // 0's carry items, 5 second barrier, 6 outputs issued, 7 wave 0's polls
  if (tid == 0) MAVG_ATRACE(0, MAVG_ANOW());
  const int pcount = a >= 0 ? (int)(jlo * TF - a) : 0;
  const long long nitem = qhi - qlo;

  auto slot = [](int g) -> int {
    if constexpr (CH) return chan_slot<CL, P>(g);
    else return stage_slot<QM>(g);
  };
  // ---- 1. the tile and the shifted tile to LDS; phase A; own / head-duty records ----
  const unsigned nb = gridDim.x;
  const unsigned bd = blockIdx.x + (unsigned)p.ahead;
  const long long ja = bd < nb ? map_tile(bd) : -1;
  // SELF (round 6, the halo-only CH form; AheadParams::self): aggregate-first records -- no phase
  // A; every tile publishes its own record from the x it holds in registers as soon as its loads
  // land, and the carry reads the records after the in-tile scan.  Every producer of a record in
  // this mode -- the tile itself, head duty, a consumer's recompute -- forms it in one order: per
  // wave, each lane's column summed over its P frames in frame order, then butterflies over the
  // lanes of the column (strides CL .. 32), then the NW waves' shares added in wave order
  // (publish_record_lds).  So the record has the same bits whoever computes it, for fp64 sums of
  // fp32 as for integer sums, and the output is the same under every schedule.
  constexpr bool kSelfOk = CH && XG;
  const bool self = kSelfOk && p.self != 0;
  const bool produce = !self && ja >= 0 && ja < p.nfull;
  // XG: the lane's x (dword column cl -- channels cl*E .. cl*E + E - 1 -- of frames j0 .. j0 + P - 1)
  const int cl = lane & (CL - 1);  // CH: the lane's dword column
  const int j0 = w * WF + (lane / CL) * P;
  uint32_t xr[XG ? P : 1];
  auto load_x = [&]() {
    if constexpr (XL >= 1) {
      xl_load<P, CL>(in, t0 + j0, cl, nframes, xr);  // every tile (transposed after the first barrier)
    } else if (tile_full) {
      const uint32_t* in32 = reinterpret_cast<const uint32_t*>(in);
#pragma unroll
      for (int i = 0; i < P; ++i) xr[i] = in32[(t0 + j0 + i) * CL + cl];
    } else {
#pragma unroll
      for (int i = 0; i < P; ++i) {
        T v[E];
#pragma unroll
        for (int e = 0; e < E; ++e) v[e] = load_elem(in, hist, t0 + j0 + i, cl * E + e, C, nframes, k, pre);
        xr[i] = CEl::put(v);
      }
    }
  };
  // XG: x first of all (round 5, in-process A/B, profiles/r05_tuning/wide/xgat_*: loaded after the
  // first barrier, or after the record carry with the in-tile scan moved there -- 118 instead of 150
  // VGPRs for 8 channels -- both slower: C = 8, k = 44100 0.570 -> 0.518 / 0.487; the tile's x
  // latency then lies on the tile's path)
  if constexpr (XG) load_x();
  // phase A's tile (its loads issued after the stage: issued first they measured 0.581 -> 0.534 for
  // 8 channels at k = 44100, profiles/r05_tuning/wide/pa_*)
  Unit<T, VE> xa[U];
  if (XG) {
    // no tile stage
  } else if (tile_full) {
    const T* src = in + t0 * C;
#pragma unroll
    for (int i = 0; i < TG / WG; ++i) {
      const int gl = slot(i * WG + tid);
      glds16<(NT & kNtLoad) != 0>(src + (long long)gl * EPG, tstage + (i * WG + wq * 64) * 16);
    }
  } else {
#pragma unroll 1
    for (int gl = tid; gl < TG; gl += WG) {
      Gr u;
#pragma unroll
      for (int i = 0; i < EPG; ++i) {
        const int e = gl * EPG + i;
        u.e[i] = load_elem(in, hist, t0 + e / C, e % C, C, nframes, k, pre);
      }
      GIO::store(reinterpret_cast<T*>(tstage + slot(gl) * 16), u);
    }
  }
  const bool stage_fast = h0 >= 0 && (h0 * C + (long long)SG * EPG) <= nframes * C;
  if (stage_fast) {
    const T* src = in + h0 * C;
    for (int j0 = 0; j0 < SG; j0 += WG) {
      const int s = j0 + tid;
      if (s < SG) glds16<(NT & kNtHalo) != 0>(src + (long long)slot(s) * EPG, sstage + (j0 + wq * 64) * 16);
    }
  } else {
#pragma unroll 1
    for (int gl = tid; gl < SG; gl += WG) {
      Gr u;
#pragma unroll
      for (int i = 0; i < EPG; ++i) {
        const int e = gl * EPG + i;
        u.e[i] = load_elem(in, hist, h0 + e / C, e % C, C, nframes, k, pre);
      }
      GIO::store(reinterpret_cast<T*>(sstage + slot(gl) * 16), u);
    }
  }
  auto share = [&](int src, const SA (&r)[C]) {
    if (lane == 0) {
#pragma unroll
      for (int c = 0; c < C; ++c) shares[(src * NW + w) * C + c] = r[c];
    }
  };
  if (produce) {  // phase A: tile t + D, default policy (its own later loads hit L2)
#pragma unroll
    for (int u = 0; u < U; ++u) xa[u] = IO::gload(in + (ja * TF + (long long)(u * WG + tid) * F) * C, false);
    SA r[C];
    wave_record<T, SA, C, F, U>(xa, r);
    share(0, r);
  }
  if (tid == 0) MAVG_ATRACE(1, MAVG_ANOW());
  // XL = 2 (with self-published records only): the columns are formed right away, since the record
  // below sums them as soon as the loads land anyway
  if constexpr (XL == 2) xl_transpose<P>(xr, cl);
  const bool own = (self || blockIdx.x < (unsigned)p.ahead) && tile < p.nfull;  // no block D slots earlier
  // SELF: the wave's share of a record in the self order, from the column values x(i) of the
  // frames of this wave's part of the tile: the lane's column sums over i in frame order, then
  // butterflies over the lanes of one column; lanes < CL hold the column totals
  auto self_share = [&](int src, auto xcol) {
    SA sc[E];
#pragma unroll
    for (int e = 0; e < E; ++e) sc[e] = (SA)0;
    xcol(sc);
#pragma unroll
    for (int e = 0; e < E; ++e)
#pragma unroll
      for (int sh = CL; sh < 64; sh <<= 1) sc[e] += __shfl_xor(sc[e], sh, 64);
    if (lane < CL)
#pragma unroll
      for (int e = 0; e < E; ++e) shares[(src * NW + w) * C + lane * E + e] = sc[e];
  };
  if (own) {
    if constexpr (kSelfOk) {
      if (self)
        self_share(1, [&](SA (&sc)[E]) {
#pragma unroll
          for (int e = 0; e < E; ++e)
#pragma unroll
            for (int i = 0; i < P; ++i) sc[e] += to_acc<SA>(CEl::get(xr[i], e));
        });
    }
    if (!self) {
      SA r[C];
      wave_record_lean<T, SA, C, F, U, WG>(in, tile, w, lane, false, r);
      share(1, r);
    }
  }
  long long jh = -1;
  if (p.xcd_remap == 1) {
    const unsigned xr = blockIdx.x & 7u, s = blockIdx.x >> 3;
    if (xr >= 1u && s < (unsigned)p.head) {
      const long long j = run_start(xr, nb) - p.head + s;
      if (j >= 0 && j < p.nfull) jh = j;
    }
  }
  // the column loads of the rare paths (head duty, recompute): frame j*TF + wave*WF + block*P + i
  const uint32_t* in32c = reinterpret_cast<const uint32_t*>(in);
  if (jh >= 0) {
    if constexpr (kSelfOk) {
      if (self)
        self_share(2, [&](SA (&sc)[E]) {
#pragma unroll 1
          for (int i = 0; i < P; ++i) {
            const uint32_t x = in32c[(jh * TF + j0 + i) * CL + cl];
#pragma unroll
            for (int e = 0; e < E; ++e) sc[e] += to_acc<SA>(CEl::get(x, e));
          }
        });
    }
    if (!self) {
      SA r[C];
      wave_record_lean<T, SA, C, F, U, WG>(in, jh, w, lane, false, r);
      share(2, r);
    }
  }
  // the carry reads one (record, channel) pair per thread: slot s = q*C + c
  // (C x fewer registers held across the scan than whole records per thread;
  // WG is a multiple of C, so a thread's channel cc is the same every round)
  const long long nslot = nitem * C;
  const int cc = tid % C;
  unsigned long long rv[NG];
  auto slot_load = [&](long long sl, unsigned long long (&v)[NG]) {
#pragma unroll
    for (int h = 0; h < NG; ++h) v[h] = gran_load(gran + (qlo * C + sl) * NG + h);
  };
  MAVG_DCHECK(qhi <= p.nfull, "wide record read range", qhi, p.nfull);
  if (!self && tid < nslot) {
    slot_load(tid, rv);
  } else {
#pragma unroll
    for (int h = 0; h < NG; ++h) rv[h] = 0ull;
  }
  __syncthreads();
  if (tid == 0) MAVG_ATRACE(2, MAVG_ANOW());
  // the three record sources (phase A, own tile, head duty), one per wave: a
  // loop, so a 2-wave workgroup (128 threads) publishes its head-duty records too
  for (int src = wq; src < 3; src += NW) {
    const long long j = src == 0 ? (produce ? ja : -1) : (src == 1 ? (own ? tile : -1) : jh);
    if (j >= 0) publish_record_lds<SA, C, NW>(gran, j, shares + (src * NW) * C, lane);
  }

  // ---- 2. the partial window before frame 0 (history / peeled head) ----
  // (CH: each thread sums its own channel cc only -- one accumulator held
  // across the scan and the carry instead of C)
  constexpr int HPC = CH ? 1 : C;
  A hp[HPC];
#pragma unroll
  for (int c = 0; c < HPC; ++c) hp[c] = (A)0;
  if (a < 0 && (hist != nullptr || pre > 0)) {
    if constexpr (CH) {
      // element e of the window before frame 0 is (frame a + e / C, channel e mod C); a
      // thread's elements are WG apart, a multiple of C: all of channel cc = tid mod C
#pragma unroll 1
      for (long long e = tid; e < -a * C; e += WG) hp[0] += to_acc<A>(load_elem(in, hist, a + e / C, cc, C, nframes, k, pre));
    } else {
#pragma unroll 1
      for (long long f = a + tid; f < 0; f += WG)
#pragma unroll
        for (int c = 0; c < C; ++c) hp[c] += to_acc<A>(load_elem(in, hist, f, c, C, nframes, k, pre));
    }
  }

  // ---- 3. the wide in-tile scan; the partial window [a, jlo T) is the x[n-k]
  //         of the tile's first pcount frames ----
  constexpr int NWD = G * 4;
  static_assert((C * sizeof(T)) % 4 == 0, "frames of whole dwords");
  auto gwords = [&](const unsigned char* base, int g, uint32_t* d) {
    const u32x4 v = *reinterpret_cast<const u32x4*>(base + stage_slot<QM>(g) * 16);
    d[0] = v[0];
    d[1] = v[1];
    d[2] = v[2];
    d[3] = v[3];
  };
  auto x_chunk = [&](int j, uint32_t (&xv)[NWD]) {
#pragma unroll
    for (int i = 0; i < G; ++i) gwords(tstage, j * G + i, xv + 4 * i);
  };
  auto xk_chunk = [&](int j, uint32_t (&xk)[NWD]) {
    const int e = (Ha - k) * C + j * CE;  // shifted-stage element of x[n-k] for the chunk's first frame
    MAVG_DCHECK(e >= 0 && e + CE <= SG * EPG, "wide ahead x[n-k] stage index", e, j);
    constexpr int kStep = C * (int)sizeof(T) / 4;
    if constexpr (kStep % 4 == 0) {
#pragma unroll
      for (int i = 0; i < G; ++i) gwords(sstage, e / EPG + i, xk + 4 * i);
    } else {
      if (p.xk_off == 0) {
#pragma unroll
        for (int i = 0; i < G; ++i) gwords(sstage, e / EPG + i, xk + 4 * i);
      } else {
        const int gs = (e - p.xk_off) / EPG;
        uint32_t flat[NWD + 4];
#pragma unroll
        for (int i = 0; i <= G; ++i) gwords(sstage, gs + i, flat + 4 * i);
        shift_words<kStep, kStep, NWD>(flat, xk, p.xk_off * (int)sizeof(T) / 4);
      }
    }
  };
  // CH: the lane's channel over its P frames, then the scan across the NB
  // lanes of the channel (chan_tile_kernel); the partial window's x[n-k] of
  // the lane's channel in hpo.
  // Stage addressing (F = 1, so Ha = k: x[n-k] of tile frame f is shifted-
  // stage frame f, the tile stage's frame f is x): element (j0 + i, cl) lies in
  // chan_slot granule j0 GPF + ((i ^ bq) << LG) + cl/4 (the key of chan_slot is
  // the lane's block bq for every i < P), i.e. at float index
  // tb[i mod NBX] + (i / NBX) * NBX * 4 GPF with a table of NBX lane offsets --
  // NBX address registers instead of the P the compiler would otherwise keep
  // live from pass 1 to pass 2.
  const uint32_t* tsf = reinterpret_cast<const uint32_t*>(tstage);
  const uint32_t* ssf = reinterpret_cast<const uint32_t*>(sstage);
  constexpr int GPFc = CL >= 4 ? CL / 4 : 1;
  constexpr int NBX = NB < P ? NB : P;
  constexpr int kFS = 4 * GPFc;  // floats per frame of the stage
  auto ch_table = [&](int lb, int bq, int (&tb)[NBX]) {
#pragma unroll
    for (int r = 0; r < NBX; ++r) tb[r] = lb + (r ^ bq) * kFS;
  };
  auto ch_idx = [&](const int (&tb)[NBX], int i) -> int { return tb[i % NBX] + (i / NBX) * NBX * kFS; };
  const int ch_lb = (j0 * GPFc + (cl >> 2)) * 4 + (cl & 3);  // frame j0 before the key
  constexpr int kGrp = 8;  // frames per scheduling group of the two passes (sched_barrier between groups)
  const int ch_bq = lane / CL;
  SA crun[E], cincl[E];  // CH: per channel of the lane's column
  A hpo[E];
#pragma unroll
  for (int e = 0; e < E; ++e) crun[e] = cincl[e] = (SA)0, hpo[e] = (A)0;
  // (PW: the wave holds frames of the partial window's x[n-k], frames < pcount -- wave-uniform,
  // so the other waves run the loop without its per-frame select)
  auto ch_pass1_loop = [&](auto pw) {
    constexpr bool PW = decltype(pw)::value;
    int tb[NBX];
    ch_table(ch_lb, ch_bq, tb);
#pragma unroll
    for (int i = 0; i < P; ++i) {
      // groups of kGrp frames the scheduler may not mix: bounded live fp64 conversions
      if (i % kGrp == 0 && i > 0) __builtin_amdgcn_sched_barrier(0);
      const int ix = ch_idx(tb, i);
      MAVG_DCHECK((ix == (chan_slot<CL, P>(((j0 + i) * CL + cl) >> 2) * 4 + (cl & 3))), "CH stage index", ix, i);
      const uint32_t xk = ssf[ix];
      uint32_t xv;
      if constexpr (XG) xv = xr[i];
      else xv = tsf[ix];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if constexpr (PW)
          if (j0 + i < pcount) hpo[e] += to_acc<A>(CEl::get(xk, e));
        crun[e] += to_acc<SA>(CEl::get(xv, e)) - to_acc<SA>(CEl::get(xk, e));
      }
    }
  };
  auto ch_pass1 = [&]() {
    static_assert(!CH || (F == 1 && NBX * (P / NBX) == P), "Ha = k: x[n-k] of tile frame f is shifted-stage frame f");
    MAVG_DCHECK(Ha == k, "CH shifted stage offset", Ha, k);
    if (pcount > wq * WF) ch_pass1_loop(std::true_type{});
    else ch_pass1_loop(std::false_type{});
#pragma unroll
    for (int e = 0; e < E; ++e) {
      cincl[e] = crun[e];
#pragma unroll
      for (int sh = CL; sh < 64; sh <<= 1) {
        SA t = shfl_up(cincl[e], sh);
        t = lane >= sh ? t : (SA)0;
        cincl[e] += t;
      }
      if (lane >= 64 - CL) tot[w * C + cl * E + e] = cincl[e];
    }
  };
  if constexpr (XL == 1) xl_transpose<P>(xr, cl);
  if constexpr (CH) ch_pass1();
  SA lx[UW][C];
#pragma unroll
  for (int uw = 0; uw < UW && !CH; ++uw) {
    const int j = uw * WG + tid;
    uint32_t xv[NWD], xk[NWD];
    x_chunk(j, xv);
    xk_chunk(j, xk);
    const int f0 = j * P;
    if (f0 < pcount) {
#pragma unroll
      for (int fr = 0; fr < P; ++fr)
        if (f0 + fr < pcount)
#pragma unroll
          for (int c = 0; c < C; ++c) hp[c] += to_acc<A>(chunk_elem<T>(xk, fr * C + c));
    }
    SA run[C];
#pragma unroll
    for (int c = 0; c < C; ++c) run[c] = (SA)0;
#pragma unroll
    for (int fr = 0; fr < P; ++fr)
#pragma unroll
      for (int c = 0; c < C; ++c)
        run[c] += to_acc<SA>(chunk_elem<T>(xv, fr * C + c)) - to_acc<SA>(chunk_elem<T>(xk, fr * C + c));
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const SA incl = wave_incl_scan(run[c]);
      lx[uw][c] = incl - run[c];
      const SA segtot = readlane(incl, 63);
      if (lane == 0) tot[(uw * NW + w) * C + c] = segtot;
    }
  }

  if (tid == 0) MAVG_ATRACE(3, MAVG_ANOW());
  // ---- 4. whole-tile carry from the records, WG (record, channel) slots per round ----
  A hq = (A)0;  // channel cc
#ifdef MAVG_AHEAD_TRACE
  unsigned polls0 = 0;
#endif
#pragma unroll 1
  for (long long sb0 = 0; sb0 < nslot; sb0 += WG) {
    const long long sl = sb0 + tid;
    const bool act = sl < nslot;
    if (sb0 != 0 || self) {
      if (act) {
        slot_load(sl, rv);
      } else {
#pragma unroll
        for (int h = 0; h < NG; ++h) rv[h] = 0ull;
      }
    }
    bool miss = false;
#pragma unroll
    for (int h = 0; h < NG; ++h) miss |= act && (rv[h] >> 32) != 1ull;
#pragma unroll 1
    for (int it = 0; __any(miss) && it < p.spin; ++it) {
#ifdef MAVG_AHEAD_STATS
      if (lane == 0) atomicAdd(reinterpret_cast<unsigned int*>(p.stats) + 1, 1u);
#endif
#ifdef MAVG_AHEAD_TRACE
      ++polls0;
#endif
      __builtin_amdgcn_s_sleep(2);
      if (miss) slot_load(sl, rv);
      miss = false;
#pragma unroll
      for (int h = 0; h < NG; ++h) miss |= act && (rv[h] >> 32) != 1ull;
    }
    // still untagged: the wave recomputes each such record from the input with
    // the producer's sequence, once per record for all the lanes of its channels
    unsigned long long mask = __ballot(miss);
#pragma unroll 1
    while (mask != 0ull) {
      const int l = __builtin_ctzll(mask);
      const long long ql = __shfl(sl, l, 64) / C;
      // one channel at a time (the producer's additions for that channel, the
      // same bits): one accumulator live instead of a whole record's C
      SA v = (SA)0;
      if (self) {
        // the self order (SELF above): this wave plays each producer wave in turn, every lane its
        // own column's element e; lane ch / E then holds channel ch's share of that wave
        if constexpr (kSelfOk) {
#pragma unroll 1
          for (int e = 0; e < E; ++e) {
            SA r = (SA)0;
#pragma unroll 1
            for (int wv = 0; wv < NW; ++wv) {
              SA sw = (SA)0;
              const long long fb = (qlo + ql) * TF + wv * WF + (lane / CL) * P;
#pragma unroll 1
              for (int i = 0; i < P; ++i) sw += to_acc<SA>(CEl::get(in32c[(fb + i) * CL + cl], e));
#pragma unroll
              for (int sh = CL; sh < 64; sh <<= 1) sw += __shfl_xor(sw, sh, 64);
              r = wv == 0 ? sw : r + sw;  // publish_record_lds: the shares in wave order
            }
            // channel cc = column cc / E, element cc mod E: lane cc / E holds that column's total
            const SA t = __shfl(r, cc / E, 64);
            if (cc % E == e) v = t;
          }
        }
      } else {
#pragma unroll 1
        for (int c = 0; c < C; ++c) {
          const SA rc = tile_record_chan_lean<T, SA, C, F, U, WG>(in, qlo + ql, c, lane);
          if (cc == c) v = rc;
        }
      }
      const bool mine = miss && sl / C == ql;
      if (mine) {
#pragma unroll
        for (int h = 0; h < NG; ++h) rv[h] = kGranTag | gran_word(v, h);
      }
#ifdef MAVG_AHEAD_STATS
      if (lane == 0) atomicAdd(reinterpret_cast<unsigned int*>(p.stats), 1u);
#endif
      mask &= ~__ballot(mine);
    }
    if (act) {
      uint32_t wd[NG];
#pragma unroll
      for (int h = 0; h < NG; ++h) wd[h] = (uint32_t)rv[h];
      hq += (A)gran_value<SA>(wd);
    }
  }
  if (tid == 0) {
    MAVG_ATRACE(4, MAVG_ANOW());
#ifdef MAVG_AHEAD_TRACE
    MAVG_ATRACE(7, polls0);
#endif
  }
  if constexpr (CH) {
    // the wave's per-channel totals by butterflies over the lanes of one channel (lane mod C
    // for the carry and the history, lane mod CL for the partial window's column sums)
    // instead of C whole-wave scans: at C = 8 the scans took 1.5 us of an 11.4-us tile
    // (the phase trace, profiles/r05_tuning/trace/)
    static_assert(64 % C == 0 && 64 % CL == 0 && CL * E == C, "channel = lane mod C; column = lane mod CL");
    A v = hp[0] + hq;  // channel cc = lane mod C
    if constexpr (E == 1) v += hpo[0];  // the column is the channel
#pragma unroll
    for (int sh = C; sh < 64; sh <<= 1) v += __shfl_xor(v, sh, 64);
    if constexpr (E > 1) {
      A hv[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        hv[e] = hpo[e];
#pragma unroll
        for (int sh = CL; sh < 64; sh <<= 1) hv[e] += __shfl_xor(hv[e], sh, 64);
      }
      // lane l < C takes channel l's column total from lane l / E (element l mod E)
      A add = (A)0;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const A t = __shfl(hv[e], lane / E, 64);
        if (lane % E == e) add = t;
      }
      v += add;
    }
    if (lane < C) hsum[w * C + lane] = v;
  } else {
    // (hp holds every channel in every thread -- the chunk scan of step 3 sums the partial
    // window's x[n-k] into it -- so these stay whole-wave scans)
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const A part = hp[c] + (cc == c ? hq : (A)0);
      const A r = readlane(wave_incl_scan(part), 63);
      if (lane == 0) hsum[w * C + c] = r;
    }
  }
  __syncthreads();
  if (tid == 0) MAVG_ATRACE(5, MAVG_ANOW());

  // ---- 5. carry + earlier segments; pass 2 rebuilt from the stages; outputs ----
  if constexpr (CH) {
    A base[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int ch = cl * E + e;
      base[e] = (A)0;
#pragma unroll
      for (int i = 0; i < NW; ++i) base[e] += hsum[i * C + ch];
#pragma unroll
      for (int i = 0; i < NW - 1; ++i)
        if (i < wq) base[e] += (A)tot[i * C + ch];
      base[e] += (A)(cincl[e] - crun[e]);
    }
    // the address table again, from values the compiler cannot prove equal to
    // pass 1's (it would keep pass 1's P addresses live across the carry)
    int lb2 = ch_lb, bq2 = ch_bq;
    asm volatile("" : "+v"(lb2), "+v"(bq2));
    if constexpr (XG) {
      // likewise x: without this the compiler keeps pass 1's fp64 conversions
      // of the P values (2 P registers) live across the carry instead of x (P)
#pragma unroll
      for (int i = 0; i < P; ++i) asm volatile("" : "+v"(xr[i]));
    }
    int tb[NBX];
    ch_table(lb2, bq2, tb);
    // each output replaces, in the shifted stage, the x[n-k] it was the last
    // read of (the same lane, the same address: no barrier); the wave then
    // reads its own frames back slot-contiguous
    uint32_t* sw = reinterpret_cast<uint32_t*>(sstage);
    // the window sum itself runs through the frames (base folded in: one add per sample fewer)
    A run[E];
#pragma unroll
    for (int e = 0; e < E; ++e) run[e] = base[e];
#pragma unroll
    for (int i = 0; i < P; ++i) {
      if (i % kGrp == 0 && i > 0) __builtin_amdgcn_sched_barrier(0);
      const int ix = ch_idx(tb, i);
      const uint32_t xk = sw[ix];
      uint32_t xv;
      if constexpr (XG) xv = xr[i];
      else xv = tsf[ix];
      T y[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        run[e] += (A)(to_acc<SA>(CEl::get(xv, e)) - to_acc<SA>(CEl::get(xk, e)));
        y[e] = to_out<T, A, DV>(run[e], p.o);
      }
      if (tile_full) {
        sw[ix] = CEl::put(y);
      } else if (t0 + j0 + i < nframes) {
#pragma unroll
        for (int e = 0; e < E; ++e) out[(t0 + j0 + i) * C + cl * E + e] = y[e];
      }
    }
    if (!tile_full) return;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    constexpr int WGR = WF * C / EPG;  // the wave's granules
    const int rg = wq * WGR;
    T* ob = out + (t0 + (long long)wq * WF) * C;
#pragma unroll
    for (int r = 0; r < WGR / 64; ++r) {
      const int s2 = rg + r * 64 + lane;
      const Gr g = GIO::load(reinterpret_cast<const T*>(sstage + s2 * 16));
      GIO::template store<(NT & kNtStore) != 0>(ob + (long long)(chan_slot<CL, P>(s2) - rg) * EPG, g);
    }
    if (tid == 0) MAVG_ATRACE(6, MAVG_ANOW());
    return;
  }
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
  T yv[UW][CE];
#pragma unroll
  for (int uw = 0; uw < UW; ++uw) {
    const int j = uw * WG + tid;
    uint32_t xv[NWD], xk[NWD];
    x_chunk(j, xv);
    xk_chunk(j, xk);
    A b[C];
#pragma unroll
    for (int c = 0; c < C; ++c) b[c] = w0[c] + (A)(readlane(ex[c], uw * NW + wq) + lx[uw][c]);
    SA run[C];
#pragma unroll
    for (int c = 0; c < C; ++c) run[c] = (SA)0;
#pragma unroll
    for (int fr = 0; fr < P; ++fr)
#pragma unroll
      for (int c = 0; c < C; ++c) {
        run[c] += to_acc<SA>(chunk_elem<T>(xv, fr * C + c)) - to_acc<SA>(chunk_elem<T>(xk, fr * C + c));
        yv[uw][fr * C + c] = to_out<T, A, DV>(b[c] + (A)run[c], p.o);
      }
  }
  if (!tile_full) {
#pragma unroll
    for (int uw = 0; uw < UW; ++uw) {
      const long long f = t0 + (long long)(uw * WG + tid) * P;
#pragma unroll
      for (int fr = 0; fr < P; ++fr)
        if (f + fr < nframes)
#pragma unroll
          for (int c = 0; c < C; ++c) out[(f + fr) * C + c] = yv[uw][fr * C + c];
    }
    return;
  }
  __syncthreads();  // every read of the tile stage is done: it takes the outputs
#pragma unroll
  for (int uw = 0; uw < UW; ++uw) {
    unsigned char* rb = tstage + ((uw * WG + wq * 64) * G) * 16;
#pragma unroll
    for (int i = 0; i < G; ++i) {
      Gr g;
#pragma unroll
      for (int e = 0; e < EPG; ++e) g.e[e] = yv[uw][i * EPG + e];
      GIO::store(reinterpret_cast<T*>(rb + out_slot(lane * G + i) * 16), g);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int uw = 0; uw < UW; ++uw) {
    const unsigned char* rb = tstage + ((uw * WG + wq * 64) * G) * 16;
    T* ob = out + (t0 + (long long)(uw * WG + wq * 64) * P) * C;
#pragma unroll
    for (int r = 0; r < G; ++r) {
      const int s = r * 64 + lane;
      const Gr g = GIO::load(reinterpret_cast<const T*>(rb + s * 16));
      GIO::template store<(NT & kNtStore) != 0>(ob + out_slot(s) * EPG, g);
    }
  }
  if (tid == 0) MAVG_ATRACE(6, MAVG_ANOW());
}

}  // namespace mavg
