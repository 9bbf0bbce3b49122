// mavg_kernels.hpp -- hand-written HIP kernels for gfx950 (CDNA4, wave64).
//
// The hot path: causal k-frame moving average over interleaved C-channel
// signals, y[f,c] = S[f,c] / k with S[f,c] = sum_{j<k} x[(f-j)C + c]
// (reference semantics: basics/profilable_moving_averager.cpp:14-37).
//
// Kernels
//   scan_kernel    single-pass STREAMING scan (replaces the reference's
//                  multi-launch recursive Blelloch / Hillis-Steele pipelines,
//                  blelloch_scan_averager.cu:40-186, hillis_steele_averager.cu:17-100).
//                  Each 256-thread workgroup owns a contiguous segment of
//                  frames and walks it chunk by chunk:
//                    d[n] = x[n] - x[n-k]          (x[n-k] from an LDS ring)
//                    W[n] = W[n-1] + d[n]          (scan of d, fp64 / int32)
//                  The scan is hierarchical: serial in-lane over F frames,
//                  64-lane DPP inclusive scan of lane totals (Blelloch flavour)
//                  or element-wise log-step __shfl_up scan (Hillis-Steele
//                  flavour), an LDS exchange of the 4*U wave-segment totals,
//                  and a register carry from chunk to chunk.  The carry into
//                  a segment is recomputed from a k-frame pre-roll instead of
//                  being propagated between workgroups, so there is no
//                  inter-workgroup communication at all (no look-back, no
//                  grid sync): 8 B/sample of HBM traffic in fp32, 4 B/sample
//                  in int16, plus k/segment of pre-roll re-read.
//   direct_kernel  LDS-tiled direct window sum (replaces profilable_sm_*.cu):
//                  a tile plus its (k-1)-frame halo is staged in LDS with
//                  16/8/4-B loads; each thread sums k frames per output.
//   naive_kernel   one thread per sample, window read from global memory
//                  (replaces profilable_parallel_averager.cu:14-23).
//   synth_kernel   counter-based synthetic input (splitmix64).
//
// Arithmetic: fp32 data accumulates in fp64 (a global fp32 prefix loses
// 1e-4..1e-1 relative); int16 data accumulates exactly in
// int32 (k <= 65535) or int64, and divides with a magic-number multiply that
// is exact truncating division (NOT the reference's float reciprocal, which
// is off on exact multiples: SURVEY.md 0.4).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mavg {

constexpr int kWG = 256;          // threads per workgroup (4 wave64s)
constexpr int kNW = kWG / 64;     // waves per workgroup

// ----------------------------------------------------------------------------
// small helpers
// ----------------------------------------------------------------------------
template <typename A> __device__ __forceinline__ A to_acc(float x) { return (A)x; }
template <typename A> __device__ __forceinline__ A to_acc(int16_t x) { return (A)x; }

// 64-lane DPP move with zero fill for invalid / masked lanes.
template <int CTRL, int RM, int BM>
__device__ __forceinline__ int32_t dpp(int32_t v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, RM, BM, false);
}
template <int CTRL, int RM, int BM>
__device__ __forceinline__ double dpp(double v) {
  int lo = __double2loint(v), hi = __double2hiint(v);
  lo = __builtin_amdgcn_update_dpp(0, lo, CTRL, RM, BM, false);
  hi = __builtin_amdgcn_update_dpp(0, hi, CTRL, RM, BM, false);
  return __hiloint2double(hi, lo);
}
template <int CTRL, int RM, int BM>
__device__ __forceinline__ int64_t dpp(int64_t v) {
  int lo = (int)(uint32_t)v, hi = (int)(uint32_t)((uint64_t)v >> 32);
  lo = __builtin_amdgcn_update_dpp(0, lo, CTRL, RM, BM, false);
  hi = __builtin_amdgcn_update_dpp(0, hi, CTRL, RM, BM, false);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// Inclusive scan across the 64 lanes of a wave: Kogge-Stone inside each
// 16-lane row (row_shr 1,2,4,8) then row_bcast:15 / row_bcast:31 to carry
// row totals across rows -- 6 DPP steps, no LDS.
template <typename A>
__device__ __forceinline__ A wave_incl_scan(A v) {
  v += dpp<0x111, 0xf, 0xf>(v);
  v += dpp<0x112, 0xf, 0xf>(v);
  v += dpp<0x114, 0xf, 0xf>(v);
  v += dpp<0x118, 0xf, 0xf>(v);
  v += dpp<0x142, 0xa, 0xf>(v);
  v += dpp<0x143, 0xc, 0xf>(v);
  return v;
}

__device__ __forceinline__ int32_t readlane(int32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ double readlane(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                          __builtin_amdgcn_readlane(__double2loint(v), l));
}
__device__ __forceinline__ int64_t readlane(int64_t v, int l) {
  uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ double shfl_up(double v, int d) { return __shfl_up(v, d, 64); }
__device__ __forceinline__ int32_t shfl_up(int32_t v, int d) { return __shfl_up(v, d, 64); }
__device__ __forceinline__ int64_t shfl_up(int64_t v, int d) {
  return (int64_t)__shfl_up((long long)v, d, 64);
}

// ----------------------------------------------------------------------------
// output conversion: window sum -> sample
// ----------------------------------------------------------------------------
struct OutParams {
  double inv_k;     // 1/k (fp32 output, int64 path estimate)
  uint32_t magic;   // int16/int32 path: q = umulhi(|S|, magic) >> shift
  int shift;
  int k;            // divisor
};

__device__ __forceinline__ float to_out_f32(double s, const OutParams& o) {
  return (float)(s * o.inv_k);
}
// exact C++ truncating division S / k for |S| < 2^31, k <= 65535
__device__ __forceinline__ int16_t to_out_i16(int32_t s, const OutParams& o) {
  uint32_t a = s < 0 ? (uint32_t)(-s) : (uint32_t)s;
  uint32_t q = (o.k == 1) ? a : (__umulhi(a, o.magic) >> o.shift);
  return (int16_t)(s < 0 ? -(int32_t)q : (int32_t)q);
}
// exact truncating division for |S| < 2^53 (large-k int16 path)
__device__ __forceinline__ int16_t to_out_i16(int64_t s, const OutParams& o) {
  int64_t a = s < 0 ? -s : s;
  int64_t q = (int64_t)((double)a * o.inv_k);
  int64_t r = a - q * (int64_t)o.k;
  while (r >= o.k) { ++q; r -= o.k; }
  while (r < 0) { --q; r += o.k; }
  return (int16_t)(s < 0 ? -q : q);
}
template <typename T, typename A>
__device__ __forceinline__ T to_out(A s, const OutParams& o);
template <> __device__ __forceinline__ float to_out<float, double>(double s, const OutParams& o) { return to_out_f32(s, o); }
template <> __device__ __forceinline__ int16_t to_out<int16_t, int32_t>(int32_t s, const OutParams& o) { return to_out_i16(s, o); }
template <> __device__ __forceinline__ int16_t to_out<int16_t, int64_t>(int64_t s, const OutParams& o) { return to_out_i16(s, o); }

// ----------------------------------------------------------------------------
// a "unit" = the F frames x C channels one lane owns per load instruction
// ----------------------------------------------------------------------------
template <typename T, int VE>
struct Unit {
  T e[VE];
};

typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
template <int BYTES> struct RawVec;
template <> struct RawVec<32> { using type = u32x8; };
template <> struct RawVec<16> { using type = u32x4; };
template <> struct RawVec<8> { using type = u32x2; };
template <> struct RawVec<4> { using type = uint32_t; };
template <> struct RawVec<2> { using type = uint16_t; };

template <typename T, int VE>
struct UnitIO {
  static constexpr int kBytes = VE * (int)sizeof(T);
  static constexpr bool kVec = (kBytes == 32 || kBytes == 16 || kBytes == 8 || kBytes == 4 || kBytes == 2);

  // p is aligned to kBytes when kVec (checked on the host for the base pointer).
  // NT: non-temporal hint (streamed-once HBM data; never used on LDS).
  template <bool NT = false>
  __device__ __forceinline__ static Unit<T, VE> load(const T* __restrict__ p) {
    Unit<T, VE> u;
    if constexpr (kVec) {
      using R = typename RawVec<kBytes>::type;
      R r;
      if constexpr (NT) r = __builtin_nontemporal_load(reinterpret_cast<const R*>(p));
      else r = *reinterpret_cast<const R*>(p);
      __builtin_memcpy(&u, &r, kBytes);
    } else {
#pragma unroll
      for (int i = 0; i < VE; ++i) u.e[i] = p[i];
    }
    return u;
  }
  template <bool NT = false>
  __device__ __forceinline__ static void store(T* __restrict__ p, const Unit<T, VE>& u) {
    if constexpr (kVec) {
      using R = typename RawVec<kBytes>::type;
      R r;
      __builtin_memcpy(&r, &u, kBytes);
      if constexpr (NT) __builtin_nontemporal_store(r, reinterpret_cast<R*>(p));
      else *reinterpret_cast<R*>(p) = r;
    } else {
#pragma unroll
      for (int i = 0; i < VE; ++i) p[i] = u.e[i];
    }
  }
};

// extract elements [O, O+VE) of the concatenation (a, b)
template <int O, typename T, int VE>
__device__ __forceinline__ Unit<T, VE> extract_at(const Unit<T, VE>& a, const Unit<T, VE>& b) {
  Unit<T, VE> r;
#pragma unroll
  for (int i = 0; i < VE; ++i) r.e[i] = (i + O < VE) ? a.e[i + O] : b.e[i + O - VE];
  return r;
}
template <int O, typename T, int VE>
__device__ __forceinline__ Unit<T, VE> extract_from(const Unit<T, VE>& a, const Unit<T, VE>& b, int o) {
  if constexpr (O + 1 >= VE) {
    return extract_at<O>(a, b);
  } else {
    if (o == O) return extract_at<O>(a, b);
    return extract_from<O + 1>(a, b, o);
  }
}
template <typename T, int VE>
__device__ __forceinline__ Unit<T, VE> extract(const Unit<T, VE>& a, const Unit<T, VE>& b, int o) {
  // o is uniform across the grid (depends only on k*C mod VE): a chain of
  // scalar compares, one static extraction taken
  return extract_from<0>(a, b, o);
}

// ----------------------------------------------------------------------------
// guarded element access: frames < 0 come from the history (the multi-GPU
// halo / the reference's zero halo, gpu_utils.h:112-123), frames >= nframes
// and frames before the history read as zero.
// ----------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T load_elem(const T* __restrict__ in, const T* __restrict__ hist,
                                       long long f, int c, int C, long long nframes, int k) {
  if (f >= 0) return f < nframes ? in[f * C + c] : (T)0;
  if (hist != nullptr && f >= -(long long)(k - 1)) return hist[(f + (k - 1)) * C + c];
  return (T)0;
}

// ----------------------------------------------------------------------------
// streaming scan kernel
// ----------------------------------------------------------------------------
struct ScanParams {
  const void* in;
  void* out;
  const void* hist;
  long long nframes;     // frames in this call
  long long seg_frames;  // frames per workgroup segment (multiple of chunk frames)
  int k;                 // window, frames
  int ring_frames;       // LDS ring size in frames (multiple of chunk frames, >= k + 2*chunk;
                         // 2*chunk when xkg)
  int pre_chunks;        // pre-roll chunks per segment (ceil((k-1)/chunk))
  int xk_off;            // (-k*C) mod VE, elements: offset of x[n-k] inside its aligned unit
  int xkg;               // 1: read x[n-k] from global memory (k too large for the LDS ring)
  int xcd_remap;         // remap mode (remap_tile): 0 identity, 1 contiguous per XCD, G>1 grouped
  OutParams o;
};

// Tile -> workgroup remaps (speed only, never correctness: blocks b and b+8
// share an XCD under the observed round-robin dispatch, cdna_hip_programming.md
// 5.5 T1).  32-bit scalar arithmetic only (the grid is < 2^31 workgroups):
// a 64-bit divide here costs ~150 SALU instructions per wave.
// mode 0: identity; 1: each XCD takes one contiguous run of nb/8 tiles
// (bijective for any nb); G = 2^g > 1: each XCD takes runs of G consecutive
// tiles and the 8 XCDs' runs are adjacent, so the whole chip works inside a
// window of 8G tiles; blocks past the last full group of 8G map to themselves.
__device__ __forceinline__ long long remap_tile(unsigned b, unsigned nb, int mode) {
  if (mode == 0) return b;
  if (mode == 1) {
    const unsigned q = nb >> 3, r = nb & 7u, x = b & 7u;
    return (long long)((x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3));
  }
  const unsigned g = (unsigned)__builtin_ctz((unsigned)mode);  // mode = G, a power of two
  const unsigned full = nb & ~((8u << g) - 1u);
  if (b >= full) return b;
  const unsigned i = b >> 3, x = b & 7u;
  return (long long)(((i >> g) << (g + 3)) + (x << g) + (i & ((1u << g) - 1u)));
}

// T: sample type; A: accumulator; C: channels; F: frames per lane unit;
// U: units per lane per chunk; HS: Hillis-Steele flavour; PD: chunks of
// global loads kept in flight in registers (1 or 2); NT: bit 0 non-temporal
// output stores, bit 1 non-temporal input loads.  p.xkg (uniform): read
// x[n-k] from global memory instead of the LDS ring (very large k).
constexpr int kNtStore = 1;
constexpr int kNtLoad = 2;
template <typename T, typename A, int C, int F, int U, bool HS, int PD = 1, int NT = 0>
__global__ __launch_bounds__(kWG) void scan_kernel(ScanParams p) {
  static_assert(PD == 1 || PD == 2, "prefetch depth 1 or 2");
  constexpr int VE = F * C;                 // elements per unit
  constexpr int CHF = kWG * F * U;          // frames per chunk
  constexpr int NSEG = U * kNW;             // wave segments per chunk
  using IO = UnitIO<T, VE>;
  using U_t = Unit<T, VE>;

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const bool xkg = p.xkg != 0;
  const int ring_elems = p.ring_frames * C;
  const int ring_bytes = (ring_elems * (int)sizeof(T) + 15) & ~15;
  T* ring = reinterpret_cast<T*>(smem);
  A* tot = reinterpret_cast<A*>(smem + ring_bytes);   // [2][NSEG][C]

  const T* __restrict__ in = static_cast<const T*>(p.in);
  T* __restrict__ out = static_cast<T*>(p.out);
  const T* __restrict__ hist = static_cast<const T*>(p.hist);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const long long nframes = p.nframes;
  const int k = p.k;
  const int R = p.ring_frames;

  const long long seg = remap_tile(blockIdx.x, gridDim.x, p.xcd_remap);
  const long long s0 = seg * p.seg_frames;
  const long long s1 = min(s0 + p.seg_frames, nframes);
  const long long p0 = s0 - (long long)p.pre_chunks * CHF;
  const int nch = p.pre_chunks + (int)((s1 - s0 + CHF - 1) / CHF);

  // ---- chunk loader into registers ----------------------------------------
  auto load_chunk = [&](U_t (&buf)[U], long long c0) {
    if (c0 >= 0 && c0 + CHF <= nframes) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long f = c0 + (long long)(u * kWG + tid) * F;
        buf[u] = IO::template load<(NT & kNtLoad) != 0>(in + f * C);
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long f = c0 + (long long)(u * kWG + tid) * F;
#pragma unroll
        for (int fr = 0; fr < F; ++fr)
#pragma unroll
          for (int c = 0; c < C; ++c)
            buf[u].e[fr * C + c] = load_elem(in, hist, f + fr, c, C, nframes, k);
      }
    }
  };
  auto ring_write = [&](const U_t (&buf)[U], int rpos) {
#pragma unroll
    for (int u = 0; u < U; ++u) IO::store(ring + (rpos + (u * kWG + tid) * F) * C, buf[u]);
  };

  // ---- prologue: zero ring, stage chunk 0, prefetch chunks 1..PD -----------
  {
    uint4 z = make_uint4(0, 0, 0, 0);
    for (int i = tid * 16; i < ring_bytes; i += kWG * 16) *reinterpret_cast<uint4*>(smem + i) = z;
  }
  // bufs[b] holds chunk ci+1 (b = (ci+1) % PD) at the top of iteration ci
  U_t buf0[U], buf1[U];
  load_chunk(buf0, p0);
  __syncthreads();
  ring_write(buf0, 0);
  if constexpr (PD == 1) {
    if (nch > 1) load_chunk(buf0, p0 + CHF);
  } else {
    if (nch > 1) load_chunk(buf1, p0 + CHF);
    if (nch > 2) load_chunk(buf0, p0 + 2LL * CHF);
  }
  __syncthreads();

  A carry[C];
#pragma unroll
  for (int c = 0; c < C; ++c) carry[c] = (A)0;
  int rpos = 0;

  // one chunk: nb holds chunk ci+1 on entry and chunk ci+1+PD on exit
  auto step = [&](const int ci, U_t (&nb)[U]) {
    const long long c0 = p0 + (long long)ci * CHF;
    const int par = ci & 1;
    // ring position (frames) of x[c0 - k]
    int kb = rpos - k;
    if (kb < 0) kb += R;

    // (a) d = x - x[n-k], per-lane / per-wave scan, wave-segment totals
    A v[U][F][C];
    A lx[U][C];  // lane exclusive prefix inside the wave segment (Blelloch flavour)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = u * kWG + tid;           // unit index in chunk
      const int q = rpos + j * F;            // ring frame position of this unit
      U_t x = IO::load(ring + q * C);
      U_t xk;
      if (xkg) {
        // x[n-k] from global memory; frames before the stream start p0 read 0
        const long long f = c0 + (long long)j * F - k;
#pragma unroll
        for (int fr = 0; fr < F; ++fr)
#pragma unroll
          for (int c = 0; c < C; ++c)
            xk.e[fr * C + c] = (f + fr < p0) ? (T)0 : load_elem(in, hist, f + fr, c, C, nframes, k);
      } else if constexpr (IO::kVec) {
        int qk = kb + j * F;
        if (qk >= R) qk -= R;
        if (p.xk_off == 0) {
          xk = IO::load(ring + qk * C);
        } else {
          // x[n-k] straddles two aligned units: read both, shift by xk_off elements
          const int e_lo = qk * C - p.xk_off;              // aligned unit holding the first element
          const int e_hi = (e_lo + VE == R * C) ? 0 : e_lo + VE;
          U_t a = IO::load(ring + e_lo);
          U_t b = IO::load(ring + e_hi);
          xk = extract(a, b, p.xk_off);
        }
      } else {
#pragma unroll
        for (int fr = 0; fr < F; ++fr) {
          int qf = kb + j * F + fr;
          if (qf >= R) qf -= R;
#pragma unroll
          for (int c = 0; c < C; ++c) xk.e[fr * C + c] = ring[qf * C + c];
        }
      }
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c)
          v[u][fr][c] = to_acc<A>(x.e[fr * C + c]) - to_acc<A>(xk.e[fr * C + c]);

      if constexpr (!HS) {
        // serial in-lane scan, then 64-lane DPP scan of the lane totals
#pragma unroll
        for (int fr = 1; fr < F; ++fr)
#pragma unroll
          for (int c = 0; c < C; ++c) v[u][fr][c] += v[u][fr - 1][c];
#pragma unroll
        for (int c = 0; c < C; ++c) {
          const A t = v[u][F - 1][c];
          const A incl = wave_incl_scan(t);
          lx[u][c] = incl - t;
          const A segtot = readlane(incl, 63);
          if (lane == 0) tot[(par * NSEG + u * kNW + w) * C + c] = segtot;
        }
      } else {
        // Hillis-Steele over the 64*F frames of the wave segment: every element
        // adds the element s frames back, s = 1, 2, 4, ..., 32F (log-step, O(n log n)).
#pragma unroll
        for (int s = 1; s < F; s <<= 1) {
          A t[F][C];
#pragma unroll
          for (int fr = 0; fr < F; ++fr)
#pragma unroll
            for (int c = 0; c < C; ++c) {
              if (fr >= s) {
                t[fr][c] = v[u][fr - s][c];
              } else {
                const A nbv = shfl_up(v[u][fr - s + F][c], 1);
                t[fr][c] = lane >= 1 ? nbv : (A)0;
              }
            }
#pragma unroll
          for (int fr = 0; fr < F; ++fr)
#pragma unroll
            for (int c = 0; c < C; ++c) v[u][fr][c] += t[fr][c];
        }
#pragma unroll
        for (int m = 1; m < 64; m <<= 1) {
#pragma unroll
          for (int fr = 0; fr < F; ++fr)
#pragma unroll
            for (int c = 0; c < C; ++c) {
              const A nbv = shfl_up(v[u][fr][c], m);
              v[u][fr][c] += lane >= m ? nbv : (A)0;
            }
        }
#pragma unroll
        for (int c = 0; c < C; ++c) {
          lx[u][c] = (A)0;
          const A segtot = readlane(v[u][F - 1][c], 63);
          if (lane == 0) tot[(par * NSEG + u * kNW + w) * C + c] = segtot;
        }
      }
    }

    // (b) stage chunk ci+1 into the ring, prefetch chunk ci+1+PD
    int rnext = rpos + CHF;
    if (rnext == R) rnext = 0;
    if (ci + 1 < nch) {
      ring_write(nb, rnext);   // xkg: a 2-chunk ring holding x only
      if (ci + 1 + PD < nch) load_chunk(nb, c0 + (long long)(1 + PD) * CHF);
    }

    // (c) one barrier per chunk
    __syncthreads();

    // (d) segment prefixes -> window sums -> outputs
    A base[U][C];
    A total[C];
#pragma unroll
    for (int c = 0; c < C; ++c) total[c] = (A)0;
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int c = 0; c < C; ++c) base[u][c] = carry[c];
#pragma unroll
    for (int s = 0; s < NSEG; ++s) {
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const A t = tot[(par * NSEG + s) * C + c];
        total[c] += t;
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (s < u * kNW + w) base[u][c] += t;
      }
    }
#pragma unroll
    for (int c = 0; c < C; ++c) carry[c] += total[c];

    if (ci >= p.pre_chunks) {
      const bool full = (c0 + CHF <= s1);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = u * kWG + tid;
        const long long f = c0 + (long long)j * F;
        U_t y;
#pragma unroll
        for (int fr = 0; fr < F; ++fr)
#pragma unroll
          for (int c = 0; c < C; ++c)
            y.e[fr * C + c] = to_out<T, A>(base[u][c] + lx[u][c] + v[u][fr][c], p.o);
        if (full) {
          IO::template store<(NT & kNtStore) != 0>(out + f * C, y);
        } else {
#pragma unroll
          for (int fr = 0; fr < F; ++fr)
            if (f + fr < s1)
#pragma unroll
              for (int c = 0; c < C; ++c) out[(f + fr) * C + c] = y.e[fr * C + c];
        }
      }
    }
    rpos = rnext;
  };

  if constexpr (PD == 1) {
    for (int ci = 0; ci < nch; ++ci) step(ci, buf0);
  } else {
    for (int ci = 0; ci < nch; ci += 2) {
      step(ci, buf1);
      if (ci + 1 < nch) step(ci + 1, buf0);
    }
  }
}

// ----------------------------------------------------------------------------
// flat-tile scan kernel: one short-lived workgroup per tile of T = 256*F*U
// frames.  The carry into the tile is rebuilt from its k-frame halo instead
// of being chained between workgroups:
//     W[t0-1] = sum_{j=t0-k}^{t0-1} x[j]            (halo reduction)
//     W[n]    = W[t0-1] + scan_{t0..n}(x[m] - x[m-k])
// The halo and the tile are staged in LDS (x[n-k] reads); the tile's own
// samples stay in registers.  Workgroups are remapped so that consecutive
// tiles run on the same XCD: the halo is the tail of the tile that XCD just
// read, an L2 hit, and all concurrently running workgroups of an XCD touch
// one contiguous window of HBM (row-buffer locality: the "flat" access
// shape that reaches 82% of HBM peak for a copy, tools/tune/membw.hip).
// Two barriers per workgroup; no inter-workgroup communication.
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
  OutParams o;
};

// GX: read x[n-k] and the halo straight from global memory (L1/L2 hits: the
// tile was just loaded by this workgroup, the halo by the previous tile's
// workgroup on the same XCD) instead of staging them in LDS; LDS then holds
// only the scan totals, so the tile size no longer depends on k.
template <typename T, typename A, int C, int F, int U, bool HS, int NT = kNtLoad | kNtStore, bool GX = false,
          int WG = kWG>
__global__ __launch_bounds__(WG) void tile_scan_kernel(TileParams p) {
  constexpr int NW = WG / 64;
  constexpr int VE = F * C;
  constexpr int TF = WG * F * U;           // tile frames
  constexpr int NSEG = U * NW;
  using IO = UnitIO<T, VE>;
  using U_t = Unit<T, VE>;

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int Hu = p.halo_units;
  const int Ha = Hu * F;                     // staged halo frames (>= k)
  const int stage_bytes = GX ? 0 : ((((Hu + U * WG + 1) * VE * (int)sizeof(T)) + 15) & ~15);
  T* stage = reinterpret_cast<T*>(smem);     // [Hu + U*256 + 1 pad] units (LDS-staged variant)
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

  // bijective XCD-aware remap (cdna_hip_programming.md 5.5 T1): blocks b and
  // b+8 share an XCD; give each XCD a contiguous run of tiles.
  const long long tile = remap_tile(blockIdx.x, gridDim.x, p.xcd_remap);
  const long long t0 = tile * TF;
  const long long h0 = t0 - Ha;              // first staged halo frame
  const bool tile_full = (t0 + TF <= nframes);

  // ---- tile -> registers (streamed once: non-temporal) and LDS ----
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
  if constexpr (!GX) {
    // ---- halo -> LDS (re-read of the previous tile's tail: L2) ----
    const bool halo_fast = h0 >= 0;
    for (int j = tid; j < Hu; j += WG) {
      const long long f = h0 + (long long)j * F;
      U_t h;
      if (halo_fast) {
        h = IO::load(in + f * C);
      } else {
#pragma unroll
        for (int fr = 0; fr < F; ++fr)
#pragma unroll
          for (int c = 0; c < C; ++c) h.e[fr * C + c] = load_elem(in, hist, f + fr, c, C, nframes, k);
      }
      IO::store(stage + j * VE, h);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) IO::store(stage + (Hu + u * WG + tid) * VE, x[u]);
    if (tid == 0) {
      U_t z;
#pragma unroll
      for (int i = 0; i < VE; ++i) z.e[i] = (T)0;
      IO::store(stage + (Hu + U * WG) * VE, z);   // pad unit (k < F reads one unit past the tile)
    }
    __syncthreads();
  }

  // ---- halo reduction: W[t0-1] = sum of the k frames before t0 ----
  {
    A hs[C];
#pragma unroll
    for (int c = 0; c < C; ++c) hs[c] = (A)0;
    if constexpr (!GX) {
      for (int i = Ha - k + tid; i < Ha; i += WG)
#pragma unroll
        for (int c = 0; c < C; ++c) hs[c] += to_acc<A>(stage[i * C + c]);
    } else {
      if (t0 - k >= 0) {
        for (int i = tid; i < k; i += WG)
#pragma unroll
          for (int c = 0; c < C; ++c) hs[c] += to_acc<A>(in[(t0 - k + i) * C + c]);
      } else {
        for (int i = tid; i < k; i += WG)
#pragma unroll
          for (int c = 0; c < C; ++c) hs[c] += to_acc<A>(load_elem(in, hist, t0 - k + i, c, C, nframes, k));
      }
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const A r = readlane(wave_incl_scan(hs[c]), 63);
      if (lane == 0) hsum[w * C + c] = r;
    }
  }

  // ---- d = x - x[n-k]; in-lane, wave and segment scans ----
  // Hillis-Steele flavour (LDS-staged): transposed ownership, lane l holds
  // frames l, l+64, ..., l+64(F-1) of its 64F-frame wave segment, so every
  // register holds 64 consecutive frames and the log-step scan runs on DPP
  // (6 steps per element, O(n log n) work) with a scalar carry across the F
  // registers; x and x[n-k] both come from the LDS stage.
  constexpr bool kHsT = HS && !GX;
  A v[U][F][C];
  A lx[U][C];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if constexpr (kHsT) {
      const int sb = (u * WG + w * 64) * F;  // tile-local first frame of this wave segment
      A run[C];
#pragma unroll
      for (int c = 0; c < C; ++c) run[c] = (A)0;
#pragma unroll
      for (int r = 0; r < F; ++r) {
        const int fl = sb + r * 64 + lane;
#pragma unroll
        for (int c = 0; c < C; ++c) {
          const A d = to_acc<A>(stage[(Ha + fl) * C + c]) - to_acc<A>(stage[(Ha + fl - k) * C + c]);
          const A incl = wave_incl_scan(d);
          v[u][r][c] = incl + run[c];
          run[c] += readlane(incl, 63);
        }
      }
#pragma unroll
      for (int c = 0; c < C; ++c) {
        lx[u][c] = (A)0;
        if (lane == 0) tot[(u * NW + w) * C + c] = run[c];
      }
      continue;
    }
    const int j = u * WG + tid;
    const int e = (Ha + j * F - k) * C;      // LDS element of x[n-k]
    U_t xk;
    if constexpr (GX) {
      const long long fk = t0 + (long long)j * F - k;    // first frame of x[n-k]
      if (fk >= 0 && tile_full) {   // full tile: the straddle read stays below t0 + TF - k + VE
        if constexpr (IO::kVec) {
          if (p.xk_off == 0) {
            xk = IO::load(in + fk * C);
          } else {
            const long long e_lo = fk * C - p.xk_off;
            U_t a = IO::load(in + e_lo);
            U_t b = IO::load(in + e_lo + VE);
            xk = extract(a, b, p.xk_off);
          }
        } else {
#pragma unroll
          for (int i = 0; i < VE; ++i) xk.e[i] = in[fk * C + i];
        }
      } else {
#pragma unroll
        for (int fr = 0; fr < F; ++fr)
#pragma unroll
          for (int c = 0; c < C; ++c) xk.e[fr * C + c] = load_elem(in, hist, fk + fr, c, C, nframes, k);
      }
    } else if constexpr (IO::kVec) {
      if (p.xk_off == 0) {
        xk = IO::load(stage + e);
      } else {
        const int e_lo = e - p.xk_off;
        U_t a = IO::load(stage + e_lo);
        U_t b = IO::load(stage + e_lo + VE);
        xk = extract(a, b, p.xk_off);
      }
    } else {
#pragma unroll
      for (int i = 0; i < VE; ++i) xk.e[i] = stage[e + i];
    }
#pragma unroll
    for (int fr = 0; fr < F; ++fr)
#pragma unroll
      for (int c = 0; c < C; ++c)
        v[u][fr][c] = to_acc<A>(x[u].e[fr * C + c]) - to_acc<A>(xk.e[fr * C + c]);
    if constexpr (!HS) {
#pragma unroll
      for (int fr = 1; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) v[u][fr][c] += v[u][fr - 1][c];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const A t = v[u][F - 1][c];
        const A incl = wave_incl_scan(t);
        lx[u][c] = incl - t;
        const A segtot = readlane(incl, 63);
        if (lane == 0) tot[(u * NW + w) * C + c] = segtot;
      }
    } else {
#pragma unroll
      for (int s = 1; s < F; s <<= 1) {
        A t[F][C];
#pragma unroll
        for (int fr = 0; fr < F; ++fr)
#pragma unroll
          for (int c = 0; c < C; ++c) {
            if (fr >= s) {
              t[fr][c] = v[u][fr - s][c];
            } else {
              const A nbv = shfl_up(v[u][fr - s + F][c], 1);
              t[fr][c] = lane >= 1 ? nbv : (A)0;
            }
          }
#pragma unroll
        for (int fr = 0; fr < F; ++fr)
#pragma unroll
          for (int c = 0; c < C; ++c) v[u][fr][c] += t[fr][c];
      }
#pragma unroll
      for (int m = 1; m < 64; m <<= 1) {
#pragma unroll
        for (int fr = 0; fr < F; ++fr)
#pragma unroll
          for (int c = 0; c < C; ++c) {
            const A nbv = shfl_up(v[u][fr][c], m);
            v[u][fr][c] += lane >= m ? nbv : (A)0;
          }
      }
#pragma unroll
      for (int c = 0; c < C; ++c) {
        lx[u][c] = (A)0;
        const A segtot = readlane(v[u][F - 1][c], 63);
        if (lane == 0) tot[(u * NW + w) * C + c] = segtot;
      }
    }
  }
  __syncthreads();

  // ---- carry: halo sum + earlier segments; outputs ----
  A base[U][C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    A w0 = (A)0;
#pragma unroll
    for (int i = 0; i < NW; ++i) w0 += hsum[i * C + c];
#pragma unroll
    for (int u = 0; u < U; ++u) base[u][c] = w0;
  }
#pragma unroll
  for (int s = 0; s < NSEG; ++s)
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const A t = tot[s * C + c];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (s < u * NW + w) base[u][c] += t;
    }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if constexpr (kHsT) {
      const long long sb = t0 + (long long)(u * WG + w * 64) * F;
#pragma unroll
      for (int r = 0; r < F; ++r) {
        const long long f = sb + r * 64 + lane;
        if (tile_full || f < nframes)
#pragma unroll
          for (int c = 0; c < C; ++c) out[f * C + c] = to_out<T, A>(base[u][c] + v[u][r][c], p.o);
      }
      continue;
    }
    const long long f = t0 + (long long)(u * WG + tid) * F;
    U_t y;
#pragma unroll
    for (int fr = 0; fr < F; ++fr)
#pragma unroll
      for (int c = 0; c < C; ++c) y.e[fr * C + c] = to_out<T, A>(base[u][c] + lx[u][c] + v[u][fr][c], p.o);
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

// ----------------------------------------------------------------------------
// look-back tile scan (windows too long for an LDS-staged halo or ring)
//
// Two launches.  Pass 1 (tile_sums_kernel) writes the sum of every whole tile
// of T = 256*F*U frames (read-only streaming, 1/2 of the algorithmic bytes for
// an fp32 pass).  Pass 2 (lookback_scan_kernel) runs the same flat,
// XCD-remapped tiles as tile_scan_kernel, but never stages the k-frame halo:
// the carry W[t0-1] (sum of the k frames before the tile) is
//   * the pass-1 sums of the whole tiles inside [t0-k, t0), plus
//   * the part of [t0-k, t0) before the first whole tile, which lies inside
//     the "shifted tile" [t0-k, t0-k+T) staged in LDS for x[n-k] anyway
//     (frames before 0 come from the history buffer instead),
// so LDS is ~2 tiles and the per-sample cost is the same for every k.
// A single-pass variant (each workgroup publishing its tile sum for later
// tiles to wait on) measured 0.25-0.37 of HBM peak: the tile just before
// is still loading when its successor needs its sum, and every agent-scope
// poll is a trip past the XCD's L2.  Pass 1 + pass 2 measured 0.42-0.51
// (DESIGN.md "Tuning").
// ----------------------------------------------------------------------------
constexpr int kLookbackHeader = 256;  // bytes of the workspace before the tile sums (reserved)

struct LookbackParams {
  const void* in;
  void* out;
  const void* hist;
  long long nframes;
  int k;
  int halo_units;   // ceil(k / F): the stage starts halo_units*F frames before the tile
  int xk_off;       // (-k*C) mod VE
  int xcd_remap;    // remap mode (remap_tile)
  const void* sums; // [ntiles][C] tile sums (A), written by tile_sums_kernel
  OutParams o;
};

// pass 1: the sum of every whole tile (per channel), reduced per lane over
// its units, then across the wave (DPP scan), then across the waves in order
template <typename T, typename A, int C, int F, int U>
__global__ __launch_bounds__(kWG) void tile_sums_kernel(const T* __restrict__ in, A* __restrict__ sums,
                                                        long long nfull, int xcd_remap) {
  constexpr int NW = kWG / 64;
  constexpr int VE = F * C;
  constexpr int TF = kWG * F * U;
  using IO = UnitIO<T, VE>;
  __shared__ A wsum[NW * C];
  const long long j = remap_tile(blockIdx.x, gridDim.x, xcd_remap);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  A ls[C];
#pragma unroll
  for (int c = 0; c < C; ++c) ls[c] = (A)0;
  if (j < nfull) {  // remap_tile is a bijection on [0, gridDim.x) = [0, nfull)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const Unit<T, VE> x = IO::template load<true>(in + (j * TF + (long long)(u * kWG + tid) * F) * C);
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) ls[c] += to_acc<A>(x.e[fr * C + c]);
    }
  }
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const A r = readlane(wave_incl_scan(ls[c]), 63);
    if (lane == 0) wsum[w * C + c] = r;
  }
  __syncthreads();
  if (tid < C && j < nfull) {
    A sm = (A)0;
#pragma unroll
    for (int q = 0; q < NW; ++q) sm += wsum[q * C + tid];
    sums[j * C + tid] = sm;
  }
}

// pass 2
template <typename T, typename A, int C, int F, int U, int NT>
__global__ __launch_bounds__(kWG) void lookback_scan_kernel(LookbackParams p) {
  constexpr int WG = kWG;
  constexpr int NW = WG / 64;
  constexpr int VE = F * C;
  constexpr int TF = WG * F * U;
  constexpr int NSEG = U * NW;
  constexpr int kStageUnits = U * WG + 1;  // the shifted tile + one unit for the misaligned x[n-k] read
  constexpr int kStageBytes = ((kStageUnits * VE * (int)sizeof(T)) + 15) & ~15;
  using IO = UnitIO<T, VE>;
  using U_t = Unit<T, VE>;

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* stage = reinterpret_cast<T*>(smem);
  A* tot = reinterpret_cast<A*>(smem + kStageBytes);  // [NSEG][C] segment totals
  A* hsum = tot + NSEG * C;                             // [NW][C] carry partials

  const T* __restrict__ in = static_cast<const T*>(p.in);
  T* __restrict__ out = static_cast<T*>(p.out);
  const T* __restrict__ hist = static_cast<const T*>(p.hist);
  const A* __restrict__ sums = static_cast<const A*>(p.sums);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int k = p.k;
  const long long nframes = p.nframes;

  const long long tile = remap_tile(blockIdx.x, gridDim.x, p.xcd_remap);
  const long long t0 = tile * TF;
  const int Ha = p.halo_units * F;
  const long long h0 = t0 - Ha;               // first staged frame (shifted tile, aligned down to F)
  const bool tile_full = (t0 + TF <= nframes);
  // whole tiles inside the window before t0: [jlo, tile); the rest of the
  // window, [a, jlo*TF), is read from the stage (a >= 0) or the history
  const long long a = t0 - k;
  const long long jlo = a >= 0 ? (a + TF - 1) / TF : 0;

  // ---- tile -> registers (streamed once) ----
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
  // ---- carry, whole-tile part (loads issued while the tile streams in) ----
  A hq[C];
#pragma unroll
  for (int c = 0; c < C; ++c) hq[c] = (A)0;
  for (long long j = jlo + tid; j < tile; j += WG)
#pragma unroll
    for (int c = 0; c < C; ++c) hq[c] += sums[j * C + c];
  // ---- shifted tile [h0, h0 + kStageUnits*F) -> LDS (read k frames back:
  //      L2 / MALL) ----
  {
    const bool fast = h0 >= 0 && h0 + (long long)kStageUnits * F <= nframes;
    for (int j = tid; j < kStageUnits; j += WG) {
      const long long f = h0 + (long long)j * F;
      U_t h;
      if (fast) {
        h = IO::load(in + f * C);
      } else {
#pragma unroll
        for (int fr = 0; fr < F; ++fr)
#pragma unroll
          for (int c = 0; c < C; ++c) h.e[fr * C + c] = load_elem(in, hist, f + fr, c, C, nframes, k);
      }
      IO::store(stage + j * VE, h);
    }
  }
  __syncthreads();

  // ---- carry W[t0-1] = partial + whole tiles ----
  {
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
      // frames [a, 0): the history; only tiles with t0 < k
      for (long long f = a + tid; f < 0; f += WG)
#pragma unroll
        for (int c = 0; c < C; ++c) hp[c] += to_acc<A>(load_elem(in, hist, f, c, C, nframes, k));
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const A r = readlane(wave_incl_scan(hp[c] + hq[c]), 63);
      if (lane == 0) hsum[w * C + c] = r;
    }
  }

  // ---- d = x - x[n-k]; in-lane, wave and segment scans ----
  A v[U][F][C];
  A lx[U][C];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int j = u * WG + tid;
    const int e = (Ha + j * F - k) * C;      // stage element of x[n-k]
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
      for (int c = 0; c < C; ++c) v[u][fr][c] = to_acc<A>(x[u].e[fr * C + c]) - to_acc<A>(xk.e[fr * C + c]);
#pragma unroll
    for (int fr = 1; fr < F; ++fr)
#pragma unroll
      for (int c = 0; c < C; ++c) v[u][fr][c] += v[u][fr - 1][c];
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const A t = v[u][F - 1][c];
      const A incl = wave_incl_scan(t);
      lx[u][c] = incl - t;
      const A segtot = readlane(incl, 63);
      if (lane == 0) tot[(u * NW + w) * C + c] = segtot;
    }
  }
  __syncthreads();

  // ---- carry + earlier segments; outputs ----
  A base[U][C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    A w0 = (A)0;
#pragma unroll
    for (int i = 0; i < NW; ++i) w0 += hsum[i * C + c];
#pragma unroll
    for (int u = 0; u < U; ++u) base[u][c] = w0;
  }
#pragma unroll
  for (int sg = 0; sg < NSEG; ++sg)
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const A t = tot[sg * C + c];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (sg < u * NW + w) base[u][c] += t;
    }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long f = t0 + (long long)(u * WG + tid) * F;
    U_t y;
#pragma unroll
    for (int fr = 0; fr < F; ++fr)
#pragma unroll
      for (int c = 0; c < C; ++c) y.e[fr * C + c] = to_out<T, A>(base[u][c] + lx[u][c] + v[u][fr][c], p.o);
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

// ----------------------------------------------------------------------------
// direct LDS-tiled kernel (small windows; replaces profilable_sm_averager.cu,
// profilable_sm_vload2.cu, profilable_sm_vload4.cu): flat tiles of
// T = 256*F*U frames, XCD-remapped like the tile scan; the tile plus its
// m*F-frame halo (m = ceil((k-1)/F)) staged in LDS with VE-element loads.
// Each lane owns F consecutive frames per unit and forms their window sums
// directly from the m+1 aligned LDS units that cover them:
//     R(t) = sum of x from the first covering unit up to frame t,
//     W[s+i] = R(s+i) - R(s+i-k)
// i.e. O(k/F) adds per output where the reference sums k values per output
// (profilable_sm_vload4.cu:84-85), and 16-B stores instead of 2-B ones.
// ----------------------------------------------------------------------------
struct DirectParams {
  const void* in;
  void* out;
  const void* hist;
  long long nframes;
  int k;
  int m;          // ceil((k-1)/F): halo units in front of every lane's own unit
  int off;        // m*F - (k-1): first window frame inside the first covering unit
  int xcd_remap;
  OutParams o;
};

template <int OFF, typename A, int F, int C>
__device__ __forceinline__ void pick_prefix(const A (&pc)[2 * F][C], A (&pre)[F][C]) {
#pragma unroll
  for (int i = 0; i < F; ++i)
#pragma unroll
    for (int c = 0; c < C; ++c) {
      constexpr int base = OFF - 1;
      pre[i][c] = (base + i < 0) ? (A)0 : pc[(base + i < 0) ? 0 : base + i][c];
    }
}

template <typename A, int F, int C>
__device__ __forceinline__ void pick_prefix_rt(int off, const A (&pc)[2 * F][C], A (&pre)[F][C]) {
  switch (off) {
    case 0: pick_prefix<0, A, F, C>(pc, pre); return;
    default: break;
  }
  if constexpr (F > 1) {
    if (off == 1) { pick_prefix<1, A, F, C>(pc, pre); return; }
  }
  if constexpr (F > 2) {
    if (off == 2) { pick_prefix<2, A, F, C>(pc, pre); return; }
    if (off == 3) { pick_prefix<3, A, F, C>(pc, pre); return; }
  }
  if constexpr (F > 4) {
    if (off == 4) { pick_prefix<4, A, F, C>(pc, pre); return; }
    if (off == 5) { pick_prefix<5, A, F, C>(pc, pre); return; }
    if (off == 6) { pick_prefix<6, A, F, C>(pc, pre); return; }
    if (off == 7) { pick_prefix<7, A, F, C>(pc, pre); return; }
  }
}

template <typename T, typename A, int C, int F, int U, int WG = kWG>
__global__ __launch_bounds__(WG) void direct_kernel(DirectParams p) {
  constexpr int VE = F * C;
  constexpr int TF = WG * F * U;
  using IO = UnitIO<T, VE>;
  using U_t = Unit<T, VE>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* stage = reinterpret_cast<T*>(smem);  // [m + U*256] units

  const T* __restrict__ in = static_cast<const T*>(p.in);
  T* __restrict__ out = static_cast<T*>(p.out);
  const T* __restrict__ hist = static_cast<const T*>(p.hist);
  const int tid = threadIdx.x;
  const int k = p.k;
  const int m = p.m;
  const long long nframes = p.nframes;

  const long long tile = remap_tile(blockIdx.x, gridDim.x, p.xcd_remap);
  const long long t0 = tile * TF;
  const long long h0 = t0 - (long long)m * F;
  const bool tile_full = (t0 + TF <= nframes);

  U_t xr[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long f = t0 + (long long)(u * WG + tid) * F;
    if (tile_full) {
      xr[u] = IO::load(in + f * C);
    } else {
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) xr[u].e[fr * C + c] = load_elem(in, hist, f + fr, c, C, nframes, k);
    }
  }
  const bool halo_fast = h0 >= 0;
  for (int j = tid; j < m; j += WG) {
    const long long f = h0 + (long long)j * F;
    U_t h;
    if (halo_fast) {
      h = IO::load(in + f * C);
    } else {
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) h.e[fr * C + c] = load_elem(in, hist, f + fr, c, C, nframes, k);
    }
    IO::store(stage + j * VE, h);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) IO::store(stage + (m + u * WG + tid) * VE, xr[u]);
  __syncthreads();

#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int q = m + u * WG + tid;  // own unit in the stage
    A own[F][C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
      A r = (A)0;
#pragma unroll
      for (int fr = 0; fr < F; ++fr) {
        r += to_acc<A>(xr[u].e[fr * C + c]);
        own[fr][c] = r;
      }
    }
    A wsum[F][C];
    if (m == 0) {  // k == 1
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) wsum[fr][c] = to_acc<A>(xr[u].e[fr * C + c]);
    } else {
      // prefix over the first two covering units (the second is the own unit when m == 1)
      const U_t u0 = IO::load(stage + (q - m) * VE);
      const U_t u1 = (m >= 2) ? IO::load(stage + (q - m + 1) * VE) : xr[u];
      A pc[2 * F][C];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        A r = (A)0;
#pragma unroll
        for (int fr = 0; fr < F; ++fr) {
          r += to_acc<A>(u0.e[fr * C + c]);
          pc[fr][c] = r;
        }
#pragma unroll
        for (int fr = 0; fr < F; ++fr) {
          r += to_acc<A>(u1.e[fr * C + c]);
          pc[F + fr][c] = r;
        }
      }
      A pre[F][C];
      pick_prefix_rt<A, F, C>(p.off, pc, pre);
      // total of the m covering units before the own unit
      A tot[C];
#pragma unroll
      for (int c = 0; c < C; ++c) tot[c] = (m >= 2) ? pc[2 * F - 1][c] : pc[F - 1][c];
      for (int j = 2; j < m; ++j) {
        const U_t uj = IO::load(stage + (q - m + j) * VE);
#pragma unroll
        for (int fr = 0; fr < F; ++fr)
#pragma unroll
          for (int c = 0; c < C; ++c) tot[c] += to_acc<A>(uj.e[fr * C + c]);
      }
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) wsum[fr][c] = tot[c] + own[fr][c] - pre[fr][c];
    }
    const long long f = t0 + (long long)(u * WG + tid) * F;
    U_t y;
#pragma unroll
    for (int fr = 0; fr < F; ++fr)
#pragma unroll
      for (int c = 0; c < C; ++c) y.e[fr * C + c] = to_out<T, A>(wsum[fr][c], p.o);
    if (tile_full) {
      IO::store(out + f * C, y);
    } else {
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
        if (f + fr < nframes)
#pragma unroll
          for (int c = 0; c < C; ++c) out[(f + fr) * C + c] = y.e[fr * C + c];
    }
  }
}

// ----------------------------------------------------------------------------
// naive kernel: one thread per sample, k reads from global memory
// (profilable_parallel_averager.cu:14-23, with the history contract instead
// of reading before the buffer).
// ----------------------------------------------------------------------------
template <typename T, typename A>
__global__ __launch_bounds__(kWG) void naive_kernel(const T* __restrict__ in, T* __restrict__ out,
                                                    const T* __restrict__ hist, long long nframes,
                                                    int C, int k, OutParams o) {
  const long long idx = (long long)blockIdx.x * kWG + threadIdx.x;
  const long long n = nframes * C;
  if (idx >= n) return;
  const long long f = idx / C;
  const int c = (int)(idx - f * C);
  A s = (A)0;
  for (int j = 0; j < k; ++j) s += to_acc<A>(load_elem(in, hist, f - j, c, C, nframes, k));
  out[idx] = to_out<T, A>(s, o);
}

// ----------------------------------------------------------------------------
// synthetic input: identical to oracle/mavg_oracle.c (oracle_synth_*)
// ----------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

template <typename T>
__global__ __launch_bounds__(kWG) void synth_kernel(T* __restrict__ out, long long n, uint64_t base, int dist) {
  const long long stride = (long long)gridDim.x * kWG;
  for (long long i = (long long)blockIdx.x * kWG + threadIdx.x; i < n; i += stride) {
    const uint64_t h = splitmix64(base + (uint64_t)i);
    if constexpr (sizeof(T) == 2) {
      out[i] = (T)(int16_t)(uint16_t)(h >> 48);
    } else {
      out[i] = dist == 1 ? (float)(h >> 40) * (1.0f / 16777216.0f) : (float)(int16_t)(uint16_t)(h >> 48);
    }
  }
}

}  // namespace mavg
