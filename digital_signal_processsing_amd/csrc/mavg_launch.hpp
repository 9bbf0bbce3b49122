// mavg_launch.hpp -- host-side launch helpers shared by the libmavg
// translation units (one TU per kernel family so the build parallelises).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdint>

#include "../../include/mavg.h"
#include "mavg_kernels.hpp"

namespace mavg {

constexpr int kMaxChannels = 8;
constexpr size_t kLdsBudget = 64 * 1024;  // per workgroup; keeps >= 2 workgroups per CU

int device_cu_count();
OutParams make_out_params(int k);

// family entry points (defined in mavg_scan_*.hip / mavg_direct.hip)
int scan_f32(int C, bool vec, bool hs, const void* in, void* out, const void* hist, long long nframes, int k,
             hipStream_t st);
int scan_i16(int C, bool vec, bool hs, const void* in, void* out, const void* hist, long long nframes, int k,
             hipStream_t st);
int scan_i16_wide(int C, bool vec, bool hs, const void* in, void* out, const void* hist, long long nframes,
                  int k, hipStream_t st);
int direct_any(int dtype, bool wide, int C, int width, const void* in, void* out, const void* hist,
               long long nframes, int k, hipStream_t st);
int naive_any(int dtype, bool wide, const void* in, void* out, const void* hist, long long nframes, int C, int k,
              hipStream_t st);

// ---- streaming scan launch ----------------------------------------------------
template <typename T, typename A, int C, int F, int U, bool HS>
int launch_scan(const void* in, void* out, const void* hist, long long nframes, int k, hipStream_t st) {
  constexpr int CHF = kWG * F * U;
  constexpr int NSEG = U * kNW;
  constexpr int VE = F * C;
  ScanParams p{};
  p.in = in;
  p.out = out;
  p.hist = hist;
  p.nframes = nframes;
  p.k = k;
  p.o = make_out_params(k);
  p.pre_chunks = (k - 1 + CHF - 1) / CHF;
  const long long ring_frames = (long long)CHF * (((long long)k + 2LL * CHF + CHF - 1) / CHF);
  const size_t tot_bytes = 2 * NSEG * C * sizeof(A);
  size_t ring_bytes = ((size_t)ring_frames * C * sizeof(T) + 15) & ~(size_t)15;
  p.xkg = 0;
  if (ring_bytes + tot_bytes > kLdsBudget) {
    p.xkg = 1;  // very large k: x[n-k] re-read from global memory, 2-chunk x ring
    ring_bytes = ((size_t)2 * CHF * C * sizeof(T) + 15) & ~(size_t)15;
    p.ring_frames = 2 * CHF;
  } else {
    p.ring_frames = (int)ring_frames;
  }
  p.xk_off = (int)((VE - ((long long)k * C) % VE) % VE);
  const size_t lds = ring_bytes + tot_bytes;

  // one segment per workgroup; aim for every CU to hold a few workgroups
  const int wg_per_cu = std::max(1, std::min(8, (int)(160 * 1024 / lds)));
  const long long target = (long long)device_cu_count() * wg_per_cu;
  long long seg = (nframes + target - 1) / target;
  seg = std::max<long long>(CHF, (seg + CHF - 1) / CHF * CHF);
  p.seg_frames = seg;
  const long long nseg = (nframes + seg - 1) / seg;
  if (nseg > 0x7fffffffLL) return MAVG_ERR_UNSUPPORTED;

  hipLaunchKernelGGL((scan_kernel<T, A, C, F, U, HS>), dim3((unsigned)nseg), dim3(kWG), lds, st, p);
  return hipGetLastError() == hipSuccess ? MAVG_OK : MAVG_ERR_HIP;
}

template <typename T, typename A, int C>
int dispatch_scan_c(bool vec, bool hs, const void* in, void* out, const void* hist, long long nframes,
                    int k, hipStream_t st) {
  constexpr int VF = (C * (int)sizeof(T) <= 16 && 16 % (C * (int)sizeof(T)) == 0) ? 16 / (C * (int)sizeof(T)) : 0;
  if constexpr (VF > 0) {
    if (vec) {
      constexpr int U = VF >= 4 ? 2 : 4;
      return hs ? launch_scan<T, A, C, VF, U, true>(in, out, hist, nframes, k, st)
                : launch_scan<T, A, C, VF, U, false>(in, out, hist, nframes, k, st);
    }
  }
  return hs ? launch_scan<T, A, C, 1, 8, true>(in, out, hist, nframes, k, st)
            : launch_scan<T, A, C, 1, 8, false>(in, out, hist, nframes, k, st);
}

template <typename T, typename A>
int dispatch_scan(int C, bool vec, bool hs, const void* in, void* out, const void* hist, long long nframes,
                  int k, hipStream_t st) {
  switch (C) {
    case 1: return dispatch_scan_c<T, A, 1>(vec, hs, in, out, hist, nframes, k, st);
    case 2: return dispatch_scan_c<T, A, 2>(vec, hs, in, out, hist, nframes, k, st);
    case 3: return dispatch_scan_c<T, A, 3>(vec, hs, in, out, hist, nframes, k, st);
    case 4: return dispatch_scan_c<T, A, 4>(vec, hs, in, out, hist, nframes, k, st);
    case 5: return dispatch_scan_c<T, A, 5>(vec, hs, in, out, hist, nframes, k, st);
    case 6: return dispatch_scan_c<T, A, 6>(vec, hs, in, out, hist, nframes, k, st);
    case 7: return dispatch_scan_c<T, A, 7>(vec, hs, in, out, hist, nframes, k, st);
    case 8: return dispatch_scan_c<T, A, 8>(vec, hs, in, out, hist, nframes, k, st);
    default: return MAVG_ERR_UNSUPPORTED;
  }
}

// ---- direct LDS-tiled launch ---------------------------------------------------
template <typename T, typename A, int C, int F>
int launch_direct(const void* in, void* out, const void* hist, long long nframes, int k, hipStream_t st) {
  DirectParams p{};
  p.in = in;
  p.out = out;
  p.hist = hist;
  p.nframes = nframes;
  p.k = k;
  p.o = make_out_params(k);
  p.halo_frames = ((k - 1) + F - 1) / F * F;
  p.tile_frames = kWG * F * 4;
  const size_t lds = (((size_t)(p.halo_frames + p.tile_frames) * C * sizeof(T)) + 15) & ~(size_t)15;
  if (lds > kLdsBudget) return MAVG_ERR_UNSUPPORTED;
  const long long nblk = (nframes + p.tile_frames - 1) / p.tile_frames;
  if (nblk > 0x7fffffffLL) return MAVG_ERR_UNSUPPORTED;
  hipLaunchKernelGGL((direct_kernel<T, A, C, F>), dim3((unsigned)nblk), dim3(kWG), lds, st, p);
  return hipGetLastError() == hipSuccess ? MAVG_OK : MAVG_ERR_HIP;
}

// width: 16 (vload4), 8 (vload2) or 0 (element loads)
template <typename T, typename A, int C>
int dispatch_direct_c(int width, const void* in, void* out, const void* hist, long long nframes, int k,
                      hipStream_t st) {
  constexpr int FB = C * (int)sizeof(T);
  constexpr int F16 = (FB <= 16 && 16 % FB == 0) ? 16 / FB : 0;
  constexpr int F8 = (FB <= 8 && 8 % FB == 0) ? 8 / FB : 0;
  if constexpr (F16 > 0) {
    if (width == 16) return launch_direct<T, A, C, F16>(in, out, hist, nframes, k, st);
  }
  if constexpr (F8 > 0) {
    if (width >= 8) return launch_direct<T, A, C, F8>(in, out, hist, nframes, k, st);
  }
  return launch_direct<T, A, C, 1>(in, out, hist, nframes, k, st);
}

template <typename T, typename A>
int dispatch_direct(int C, int width, const void* in, void* out, const void* hist, long long nframes, int k,
                    hipStream_t st) {
  switch (C) {
    case 1: return dispatch_direct_c<T, A, 1>(width, in, out, hist, nframes, k, st);
    case 2: return dispatch_direct_c<T, A, 2>(width, in, out, hist, nframes, k, st);
    case 3: return dispatch_direct_c<T, A, 3>(width, in, out, hist, nframes, k, st);
    case 4: return dispatch_direct_c<T, A, 4>(width, in, out, hist, nframes, k, st);
    case 5: return dispatch_direct_c<T, A, 5>(width, in, out, hist, nframes, k, st);
    case 6: return dispatch_direct_c<T, A, 6>(width, in, out, hist, nframes, k, st);
    case 7: return dispatch_direct_c<T, A, 7>(width, in, out, hist, nframes, k, st);
    case 8: return dispatch_direct_c<T, A, 8>(width, in, out, hist, nframes, k, st);
    default: return MAVG_ERR_UNSUPPORTED;
  }
}

template <typename T, typename A>
int launch_naive(const void* in, void* out, const void* hist, long long nframes, int C, int k, hipStream_t st) {
  const long long n = nframes * C;
  const long long nblk = (n + kWG - 1) / kWG;
  if (nblk > 0x7fffffffLL) return MAVG_ERR_UNSUPPORTED;
  hipLaunchKernelGGL((naive_kernel<T, A>), dim3((unsigned)nblk), dim3(kWG), 0, st, static_cast<const T*>(in),
                     static_cast<T*>(out), static_cast<const T*>(hist), nframes, C, k, make_out_params(k));
  return hipGetLastError() == hipSuccess ? MAVG_OK : MAVG_ERR_HIP;
}

}  // namespace mavg
