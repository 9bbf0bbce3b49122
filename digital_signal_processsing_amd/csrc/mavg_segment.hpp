// mavg_segment.hpp -- the segment-streaming scan (scan_kernel).
#pragma once

#include "mavg_device.hpp"

namespace mavg {

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
  int pre;               // frames in front of `in` that are readable signal (load_elem)
  int eio;               // frame-unit launch on element-aligned pointers (UnitIO::gload)
  OutParams o;
};

// T: sample type; A: accumulator; C: channels; F: frames per lane unit;
// U: units per lane per chunk; HS: Hillis-Steele flavour; PD: chunks of
// global loads kept in flight in registers (1 or 2); NT: bit 0 non-temporal
// output stores, bit 1 non-temporal input loads.  p.xkg (uniform): read
// x[n-k] from global memory instead of the LDS ring (very large k).
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
  const int pre = p.pre;
  const bool eio = F == 1 && p.eio != 0;

  const long long seg = remap_tile(blockIdx.x, gridDim.x, p.xcd_remap);
  MAVG_DCHECK(seg >= 0 && seg < (long long)gridDim.x && seg * p.seg_frames < nframes, "segment index", seg, gridDim.x);
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
        buf[u] = IO::template gload<(NT & kNtLoad) != 0>(in + f * C, eio);
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long f = c0 + (long long)(u * kWG + tid) * F;
#pragma unroll
        for (int fr = 0; fr < F; ++fr)
#pragma unroll
          for (int c = 0; c < C; ++c)
            buf[u].e[fr * C + c] = load_elem(in, hist, f + fr, c, C, nframes, k, pre);
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
            xk.e[fr * C + c] = (f + fr < p0) ? (T)0 : load_elem(in, hist, f + fr, c, C, nframes, k, pre);
      } else if constexpr (IO::kVec) {
        int qk = kb + j * F;
        if (qk >= R) qk -= R;
        MAVG_DCHECK(qk >= 0 && qk + F <= R, "segment ring x[n-k]", qk, R);
        if (p.xk_off == 0) {
          xk = IO::load(ring + qk * C);
        } else {
          // x[n-k] straddles two aligned units: read both, shift by xk_off elements
          const int e_lo = qk * C - p.xk_off;              // aligned unit holding the first element
          const int e_hi = (e_lo + VE == R * C) ? 0 : e_lo + VE;
          U_t a = IO::load_whole(ring + e_lo);
          U_t b = IO::load_whole(ring + e_hi);
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

    // (d) segment prefixes -> window sums -> outputs: lane i holds wave
    // segment i's total, one exclusive wave scan gives every prefix, each unit
    // reads its own with a uniform readlane (mavg_tile.hpp, same idea)
    static_assert(NSEG <= 64, "segment totals are scanned across one wave");
    const int wu = __builtin_amdgcn_readfirstlane(w);
    A base[U][C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const A tv = lane < NSEG ? tot[(par * NSEG + lane) * C + c] : (A)0;
      const A incl = wave_incl_scan(tv);
      const A ex = incl - tv;
#pragma unroll
      for (int u = 0; u < U; ++u) base[u][c] = carry[c] + readlane(ex, u * kNW + wu);
      carry[c] += readlane(incl, NSEG - 1);
    }

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
          IO::template gstore<(NT & kNtStore) != 0>(out + f * C, y, eio);
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

}  // namespace mavg
