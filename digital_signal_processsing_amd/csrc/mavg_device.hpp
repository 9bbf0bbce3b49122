// mavg_device.hpp -- device building blocks shared by the kernels (gfx950, wave64):
// accumulator conversion, DPP wave scans, output conversion, 16-B lane units,
// guarded element access, the XCD-aware tile mapping.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

// Debug build (make -C csrc debug -> libmavg_debug.so): device bounds checks on LDS
// stage indices, x[n-k] extractions, tile indices and record slots; a failed
// check prints (what, block, thread, two values) and traps.  Compiled out of
// the release library.
#ifdef MAVG_DEBUG
#define MAVG_DCHECK(cond, what, a, b)                                                                   \
  do {                                                                                                \
    if (!(cond)) {                                                                                    \
      printf("mavg debug check failed: %s (block %u thread %u: %lld, %lld)\n", what, blockIdx.x,      \
             threadIdx.x, (long long)(a), (long long)(b));                                            \
      __builtin_trap();                                                                               \
    }                                                                                                 \
  } while (0)
#else
#define MAVG_DCHECK(cond, what, a, b) ((void)0)
#endif

namespace mavg {

constexpr int kWG = 256;          // threads per workgroup (4 wave64s)
constexpr int kNW = kWG / 64;     // waves per workgroup

// ----------------------------------------------------------------------------
// small helpers
// ----------------------------------------------------------------------------
template <typename A> __device__ __forceinline__ A to_acc(float x) { return (A)x; }
template <typename A> __device__ __forceinline__ A to_acc(int16_t x) { return (A)x; }

// 64-lane DPP move with zero fill for invalid / masked lanes: old = 0 for the rows row_mask
// leaves unwritten, bound_ctrl for source lanes outside the row (with full masks every lane is
// then written, so the compiler drops the zero init of the destination)
template <int CTRL, int RM, int BM>
__device__ __forceinline__ int32_t dpp(int32_t v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, RM, BM, true);
}
template <int CTRL, int RM, int BM>
__device__ __forceinline__ double dpp(double v) {
  int lo = __double2loint(v), hi = __double2hiint(v);
  lo = __builtin_amdgcn_update_dpp(0, lo, CTRL, RM, BM, true);
  hi = __builtin_amdgcn_update_dpp(0, hi, CTRL, RM, BM, true);
  return __hiloint2double(hi, lo);
}
template <int CTRL, int RM, int BM>
__device__ __forceinline__ int64_t dpp(int64_t v) {
  int lo = (int)(uint32_t)v, hi = (int)(uint32_t)((uint64_t)v >> 32);
  lo = __builtin_amdgcn_update_dpp(0, lo, CTRL, RM, BM, true);
  hi = __builtin_amdgcn_update_dpp(0, hi, CTRL, RM, BM, true);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// 4 x 4 dword transpose inside each lane quad (lanes 4j .. 4j + 3), two DPP quad_perm stages:
// on entry lane q holds a[e] = element (q, e), on exit a[f] = element (f, q).  Stage s (1, 2)
// swaps the off-diagonal halves of the 2s x 2s blocks: per pair (e, e | s) a lane sends the value
// its partner q ^ s keeps and takes the partner's (one cndmask, one DPP move, one cndmask).
// (round 6: 16-B frame loads turned into the channel-per-lane columns, mavg_wide.hpp XL)
__device__ __forceinline__ void quad_transpose4(uint32_t (&a)[4], int q) {
#pragma unroll
  for (int s = 1; s <= 2; s <<= 1) {
    const bool hi_lane = (q & s) != 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (e & s) continue;
      // value selects only (a select of the element to write made the compiler index the array
      // through scratch)
      const uint32_t lo = a[e], hi = a[e | s];
      const uint32_t send = hi_lane ? lo : hi;
      const uint32_t got = s == 1 ? (uint32_t)dpp<0xB1, 0xf, 0xf>((int32_t)send)    // quad_perm [1,0,3,2]
                                  : (uint32_t)dpp<0x4E, 0xf, 0xf>((int32_t)send);   // quad_perm [2,3,0,1]
      a[e] = hi_lane ? got : lo;
      a[e | s] = hi_lane ? hi : got;
    }
  }
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

// N independent inclusive scans, step by step across the N values (each value sees the same
// six additions in the same order as wave_incl_scan): the DPP moves of one value fill the wait
// states after the previous value's add instead of s_nops on one dependent chain
template <typename A, int N>
__device__ __forceinline__ void wave_incl_scan_n(A (&v)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += dpp<0x111, 0xf, 0xf>(v[i]);
  __builtin_amdgcn_sched_barrier(0);  // keep the steps apart: the scheduler would chain them
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += dpp<0x112, 0xf, 0xf>(v[i]);
  __builtin_amdgcn_sched_barrier(0);  // keep the steps apart: the scheduler would chain them
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += dpp<0x114, 0xf, 0xf>(v[i]);
  __builtin_amdgcn_sched_barrier(0);  // keep the steps apart: the scheduler would chain them
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += dpp<0x118, 0xf, 0xf>(v[i]);
  __builtin_amdgcn_sched_barrier(0);  // keep the steps apart: the scheduler would chain them
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += dpp<0x142, 0xa, 0xf>(v[i]);
  __builtin_amdgcn_sched_barrier(0);  // keep the steps apart: the scheduler would chain them
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += dpp<0x143, 0xc, 0xf>(v[i]);
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
  double inv_k;     // 1/k (fp32 output)
  double inv_up;    // (1/k)(1 + ~2^-50), rounded: the int16 quotient estimate (to_out_i16)
  int k;            // divisor
  uint32_t magic;   // to_out_i16_magic: q = umulhi(|S|, magic) >> shift (k <= 65535)
  int shift;
};

__device__ __forceinline__ float to_out_f32(double s, const OutParams& o) {
  return (float)(s * o.inv_k);
}
// Exact C++ truncating division S / k for the int16 output: |S| <= 32768 k
// (a sum of k int16 samples, so |S / k| <= 2^15) and k < 2^33.  With
// inv_up = fl(fl(1/k) (1 + 2^-50)) the product P = fl(S inv_up) satisfies
// S/k < P < (S/k)(1 + 2^-48) for S > 0 (every rounding factor lies within
// 2^-52 of 1, the bias is 2^-50): an exact quotient q stays in [q, q + 2^-33)
// and a non-integral one q + f (1/k <= f <= 1 - 1/k, 1/k > 2^-33) in
// (q + f, q + f + 2^-33) -- truncation gives q either way; S < 0 mirrors it
// (the product's sign is S's, v_cvt_i32_f64 truncates toward zero).  Three
// full-rate VALU ops per sample (cvt, mul, cvt), no branches and no sign
// fix-ups.  tests/test_division.py checks the rule against exact integer
// division at every k <= 65535 and sampled k up to 2^31.
__device__ __forceinline__ int16_t to_out_i16(int32_t s, const OutParams& o) {
  return (int16_t)(int32_t)((double)s * o.inv_up);
}
// The integer alternative for the int32 path: an unsigned magic-number
// multiply on |S| (exact for |S| < 2^31, k <= 65535: the magic is
// floor(2^(31+l) / k) + 1 with l = ceil(log2 k)), then the sign.
__device__ __forceinline__ int16_t to_out_i16_magic(int32_t s, const OutParams& o) {
  const uint32_t a = s < 0 ? (uint32_t)(-s) : (uint32_t)s;
  const uint32_t q = o.k == 1 ? a : (__umulhi(a, o.magic) >> o.shift);
  return (int16_t)(s < 0 ? -(int32_t)q : (int32_t)q);
}
// int64 path (k > 65535): |S| <= 32768 k < 2^47 converts exactly from its
// two halves, then the same product
__device__ __forceinline__ int16_t to_out_i16(int64_t s, const OutParams& o) {
  const double sd = (double)(int32_t)(s >> 32) * 4294967296.0 + (double)(uint32_t)s;  // exact
  return (int16_t)(int32_t)(sd * o.inv_up);
}
// DV (int32 int16 path only): 0 = the fp64 product, 1 = the magic multiply
template <typename T, typename A, int DV = 0>
__device__ __forceinline__ T to_out(A s, const OutParams& o) {
  if constexpr (sizeof(T) == 4) {
    return to_out_f32(s, o);
  } else if constexpr (DV == 1 && sizeof(A) == 4) {
    return to_out_i16_magic(s, o);
  } else {
    return to_out_i16(s, o);
  }
}

// ----------------------------------------------------------------------------
// a "unit" = the F frames x C channels one lane owns per load instruction
// ----------------------------------------------------------------------------
template <typename T, int VE>
struct Unit {
  T e[VE];
};

typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
template <int BYTES> struct RawVec;
template <> struct RawVec<64> { using type = u32x16; };  // 2 frames of 8 fp32 channels (4 x 16-B accesses)
template <> struct RawVec<32> { using type = u32x8; };
template <> struct RawVec<16> { using type = u32x4; };
template <> struct RawVec<8> { using type = u32x2; };
template <> struct RawVec<4> { using type = uint32_t; };
template <> struct RawVec<2> { using type = uint16_t; };

template <typename T, int VE>
struct UnitIO {
  static constexpr int kBytes = VE * (int)sizeof(T);
  static constexpr bool kVec = (kBytes == 64 || kBytes == 32 || kBytes == 16 || kBytes == 8 || kBytes == 4 || kBytes == 2);

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
  // The two aligned LDS units an extraction (below) reads from.  Volatile
  // keeps each a whole 16-B load: an extraction at o >= 1 never reads a.e[0]
  // (nor b.e[VE-1]), and with plain loads the compiler narrows the pair into a
  // misaligned ds_read_b96 + ds_read_u16, which bank-conflict (int16 mono at
  // k = 1023 or 1020: 12 conflict cycles per wave, 0.725 of peak against 0.81
  // at k = 1024; profiles/r02_tuning/r02_odd, pmc_odd).  An empty asm that
  // pins the registers instead forces a wait after every load (0.68).
  __device__ __forceinline__ static Unit<T, VE> load_whole(const T* p) {  // LDS only
    Unit<T, VE> u;
    if constexpr (kVec) {
      using R = typename RawVec<kBytes>::type;
      const R r = *(const volatile __attribute__((address_space(3))) R*)p;  // p points into LDS
      __builtin_memcpy(&u, &r, kBytes);
    } else {
#pragma unroll
      for (int i = 0; i < VE; ++i) u.e[i] = p[i];
    }
    return u;
  }
  // Global-memory forms.  eio (uniform): the pointer is only element-aligned
  // (a frame-unit launch on a misaligned view, mavg_api.hip), so a
  // multi-element unit moves as element accesses instead of one vector access.
  template <bool NT = false>
  __device__ __forceinline__ static Unit<T, VE> gload(const T* __restrict__ p, bool eio) {
    if constexpr (kVec && VE > 1) {
      if (eio) {
        Unit<T, VE> u;
#pragma unroll
        for (int i = 0; i < VE; ++i) u.e[i] = p[i];
        return u;
      }
    }
    return load<NT>(p);
  }
  template <bool NT = false>
  __device__ __forceinline__ static void gstore(T* __restrict__ p, const Unit<T, VE>& u, bool eio) {
    if constexpr (kVec && VE > 1) {
      if (eio) {
#pragma unroll
        for (int i = 0; i < VE; ++i) p[i] = u.e[i];
        return;
      }
    }
    store<NT>(p, u);
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
// and frames before the history read as zero.  `pre` > 0 (the body launch
// after a peeled misaligned head, mavg_api.hip): frames [-pre, 0) are the
// head, readable in front of `in`, and only frames before -pre come from
// `hist` (which the host then offsets by pre frames).
// ----------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T load_elem(const T* __restrict__ in, const T* __restrict__ hist,
                                       long long f, int c, int C, long long nframes, int k, int pre) {
  if (f >= -(long long)pre) return f < nframes ? in[f * C + c] : (T)0;
  if (hist != nullptr && f >= -(long long)(k - 1)) return hist[(f + (k - 1)) * C + c];
  return (T)0;
}

// ----------------------------------------------------------------------------
// tile -> workgroup mapping
// ----------------------------------------------------------------------------
// Tile -> workgroup remaps (speed only, never correctness: blocks b and b+8
// share an XCD under the observed round-robin dispatch, cdna_hip_programming.md
// 5.5 T1).  32-bit scalar arithmetic only (the grid is < 2^31 workgroups):
// a 64-bit divide here costs ~150 SALU instructions per wave.
// mode 0: identity; 1: each XCD takes one contiguous run of nb/8 tiles
// (bijective for any nb); G > 1: each XCD takes runs of G consecutive tiles
// and the 8 XCDs' runs are adjacent (a "period" of 8G tiles), so the whole
// chip works inside a window of 8G tiles and tile t + 8G runs on t's XCD;
// blocks past the last full period map to themselves.  G a power of two:
// shifts; otherwise one 32-bit divide per call.
__device__ __forceinline__ long long remap_tile(unsigned b, unsigned nb, int mode) {
  if (mode == 0) return b;
  if (mode == 1) {
    const unsigned q = nb >> 3, r = nb & 7u, x = b & 7u;
    return (long long)((x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3));
  }
  const unsigned G = (unsigned)mode;
  const unsigned i = b >> 3, x = b & 7u;
  if ((G & (G - 1u)) == 0u) {
    const unsigned g = (unsigned)__builtin_ctz(G);
    const unsigned full = nb & ~((8u << g) - 1u);
    if (b >= full) return b;
    return (long long)(((i >> g) << (g + 3)) + (x << g) + (i & (G - 1u)));
  }
  const unsigned full = nb - nb % (8u * G);
  if (b >= full) return b;
  const unsigned per = i / G;
  return (long long)(per * 8u * G + x * G + (i - per * G));
}

// One 16-B LDS-DMA load per lane (global_load_lds_dwordx4): lane l's 16 bytes
// land at lds_wave + 16 l; lds_wave must be wave-uniform (it goes to M0).
// NT: non-temporal (aux = 2).
template <bool NT = false>
__device__ __forceinline__ void glds16(const void* g, void* lds_wave) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave, 16, 0, NT ? 2 : 0);
}

// non-temporal (streamed-once) policy bits of the NT template parameters
constexpr int kNtStore = 1;
constexpr int kNtLoad = 2;
// tile scan only: nt loads for the part of the tile that no later tile's
// halo re-reads (the last halo-size frames stay plain, so the next tile finds
// them in L2), and nt loads for the halo itself (its last use)
constexpr int kNtSplit = 4;
constexpr int kNtHalo = 8;
// look-ahead scan only: phase A's loads of tile t + D non-temporal (very long
// windows: the prefetched tile then leaves the XCD's L2 before the window's
// lines do; its own workgroup's later loads are served by L2 or the MALL)
constexpr int kNtPhaseA = 16;

}  // namespace mavg
