// mavg_direct.hpp -- the direct LDS-tiled window sum (direct_kernel).
#pragma once

#include "mavg_device.hpp"

namespace mavg {

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
  int pre;        // frames in front of `in` that are readable signal (load_elem)
  int eio;        // frame-unit launch on element-aligned pointers (UnitIO::gload)
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

// NT: non-temporal policy bits (mavg_device.hpp): kNtLoad the tile's loads,
// kNtHalo the halo's, kNtStore the output stores
template <typename T, typename A, int C, int F, int U, int WG = kWG, int NT = 0>
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
  const int pre = p.pre;
  const bool eio = F == 1 && p.eio != 0;

  const long long tile = remap_tile(blockIdx.x, gridDim.x, p.xcd_remap);
  const long long t0 = tile * TF;
  const long long h0 = t0 - (long long)m * F;
  MAVG_DCHECK(tile >= 0 && tile < (long long)gridDim.x && t0 < nframes, "direct tile index", tile, gridDim.x);
  const bool tile_full = (t0 + TF <= nframes);

  U_t xr[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long f = t0 + (long long)(u * WG + tid) * F;
    if (tile_full) {
      xr[u] = IO::template gload<(NT & kNtLoad) != 0>(in + f * C, eio);
    } else {
#pragma unroll
      for (int fr = 0; fr < F; ++fr)
#pragma unroll
        for (int c = 0; c < C; ++c) xr[u].e[fr * C + c] = load_elem(in, hist, f + fr, c, C, nframes, k, pre);
    }
  }
  const bool halo_fast = h0 >= 0;
  for (int j = tid; j < m; j += WG) {
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
        MAVG_DCHECK(q - m + j >= 0 && q - m + j < m + U * WG, "direct stage unit", q - m + j, m);
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
