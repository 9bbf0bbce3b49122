// mavg_misc.hpp -- the naive per-sample kernel and the synthetic-input generator.
#pragma once

#include "mavg_device.hpp"

namespace mavg {

// ----------------------------------------------------------------------------
// naive kernel: one thread per sample, k reads from global memory
// (profilable_parallel_averager.cu:14-23, with the history contract instead
// of reading before the buffer).
// ----------------------------------------------------------------------------
template <typename T, typename A>
__global__ __launch_bounds__(1024) void naive_kernel(const T* __restrict__ in, T* __restrict__ out,
                                                     const T* __restrict__ hist, long long nframes,
                                                     int C, int k, OutParams o) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long n = nframes * C;
  if (idx >= n) return;
  const long long f = idx / C;
  const int c = (int)(idx - f * C);
  A s = (A)0;
  for (int j = 0; j < k; ++j) s += to_acc<A>(load_elem(in, hist, f - j, c, C, nframes, k, 0));
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

// dist 2 (oracle synth_f32_dist2): an Irwin-Hall integer from the four 14-bit
// fields, times fl64(1/3000), times 2^-s (s from the 5 bits above), rounded to
// fp32 -- each step one correctly rounded IEEE operation (no add, so nothing
// to contract into an fma), so host and device agree bit for bit
__device__ __forceinline__ float synth_f32_dist2(uint64_t h) {
  const long long i = (long long)(h & 0x3fffu) + (long long)((h >> 14) & 0x3fffu) +
                      (long long)((h >> 28) & 0x3fffu) + (long long)((h >> 42) & 0x3fffu) - 32766;
  const int b = (int)((h >> 56) & 31u);
  const int s = b < 8 ? 0 : b - 8;
  const double p = __longlong_as_double((long long)(1023 - s) << 52);  // 2^-s, exactly
  const double v = (double)i * (1.0 / 3000.0);
  return (float)(v * p);
}

template <typename T>
__global__ __launch_bounds__(kWG) void synth_kernel(T* __restrict__ out, long long n, uint64_t base, int dist) {
  const long long stride = (long long)gridDim.x * kWG;
  for (long long i = (long long)blockIdx.x * kWG + threadIdx.x; i < n; i += stride) {
    const uint64_t h = splitmix64(base + (uint64_t)i);
    if constexpr (sizeof(T) == 2) {
      out[i] = (T)(int16_t)(uint16_t)(h >> 48);
    } else {
      out[i] = dist == 1   ? (float)(h >> 40) * (1.0f / 16777216.0f)
               : dist == 2 ? synth_f32_dist2(h)
                           : (float)(int16_t)(uint16_t)(h >> 48);
    }
  }
}

// ----------------------------------------------------------------------------
// HBM calibration copy (mavg_stream_copy): one 16-B non-temporal load and
// store per thread over a flat grid -- the fastest copy shape measured
// (tools/tune/membw.hip)
// ----------------------------------------------------------------------------
template <typename V>
__global__ __launch_bounds__(kWG) void stream_copy_kernel(const V* __restrict__ in, V* __restrict__ out, long long n) {
  const long long i = (long long)blockIdx.x * kWG + threadIdx.x;
  if (i < n) __builtin_nontemporal_store(__builtin_nontemporal_load(in + i), out + i);
}

}  // namespace mavg
