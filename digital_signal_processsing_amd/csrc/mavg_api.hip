// mavg_api.hip -- C ABI of libmavg (declared in include/mavg.h).
//
// Host-side dispatch: validates arguments (the reference never validates
// grade or channels, SURVEY.md 8b "Errors"), resolves the algorithm, sizes the
// launch and enqueues exactly one kernel on the caller's stream.  No
// allocation, no synchronisation, no exit(): the reference's CUDA_CHECK
// (gpu_utils.h:10-18) becomes a returned status.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "mavg_launch.hpp"

using namespace mavg;

namespace {

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

size_t elem_size(int dtype) { return dtype == MAVG_F32 ? 4 : 2; }

// frames per 16-B unit for (dtype, C), 0 if C*elem does not divide 16
int vec_frames(int dtype, int C) {
  const int eb = (int)elem_size(dtype);
  const int fb = eb * C;
  if (fb > 16 || 16 % fb != 0) return 0;
  return 16 / fb;
}

bool is_vec_algo(int algo) {
  return algo == MAVG_ALGO_BLELLOCH || algo == MAVG_ALGO_HILLIS || algo == MAVG_ALGO_DIRECT ||
         algo == MAVG_ALGO_DIRECT_VEC2;
}

int validate(size_t n, int C, int k, int dtype, int algo) {
  if (dtype != MAVG_I16 && dtype != MAVG_F32) return MAVG_ERR_INVALID_ARG;
  if (algo < MAVG_ALGO_AUTO || algo > MAVG_ALGO_NAIVE) return MAVG_ERR_INVALID_ARG;
  if (C < 1 || k < 1) return MAVG_ERR_INVALID_ARG;
  if (n % (size_t)C != 0) return MAVG_ERR_INVALID_ARG;
  if (C > kMaxChannels && algo != MAVG_ALGO_AUTO && algo != MAVG_ALGO_NAIVE) return MAVG_ERR_UNSUPPORTED;
  if (n / (size_t)C > (size_t)0x3fffffffffffffffULL) return MAVG_ERR_UNSUPPORTED;
  return MAVG_OK;
}

}  // namespace

extern "C" {

int mavg_abi_version(void) { return MAVG_ABI_VERSION; }

const char* mavg_strerror(int status) {
  switch (status) {
    case MAVG_OK: return "ok";
    case MAVG_ERR_INVALID_ARG: return "invalid argument";
    case MAVG_ERR_UNSUPPORTED: return "unsupported configuration";
    case MAVG_ERR_MISALIGNED: return "pointer not 16-byte aligned for a vectorized algorithm";
    case MAVG_ERR_WORKSPACE: return "workspace too small";
    case MAVG_ERR_HIP: return "HIP runtime error";
    default: return "unknown status";
  }
}

const char* mavg_algo_name(int algo) {
  switch (algo) {
    case MAVG_ALGO_AUTO: return "auto";
    case MAVG_ALGO_BLELLOCH: return "blelloch";
    case MAVG_ALGO_BLELLOCH_SCALAR: return "blelloch_scalar";
    case MAVG_ALGO_HILLIS: return "hillis";
    case MAVG_ALGO_HILLIS_SCALAR: return "hillis_scalar";
    case MAVG_ALGO_DIRECT: return "direct";
    case MAVG_ALGO_DIRECT_VEC2: return "direct_vec2";
    case MAVG_ALGO_DIRECT_SCALAR: return "direct_scalar";
    case MAVG_ALGO_NAIVE: return "naive";
    default: return "invalid";
  }
}

// AUTO: the Blelloch scan family at every window (flat tiles with the tile
// shape chosen by dispatch_scan_f; O(1) work per output for any k).  The
// direct kernel is kept for MAVG_ALGO_DIRECT*: since the tile scan's carry
// became a wave scan of the segment totals, tiles beat it even at k <= 9
// (k=7, 2^28 samples: fp32 0.821 vs 0.797 of HBM peak, int16 0.795 vs 0.761,
// tools/tune/tune_scan.hip).  Both move 1.00x the algorithmic bytes on HBM.
// More than kMaxChannels channels: only the naive kernel (runtime C) applies.
int mavg_resolve_algo(size_t n_samples, int channels, int grade, int dtype, int algo) {
  (void)n_samples;
  (void)dtype;
  (void)grade;
  if (algo != MAVG_ALGO_AUTO) return algo;
  if (channels > kMaxChannels) return MAVG_ALGO_NAIVE;
  return MAVG_ALGO_BLELLOCH;
}

int mavg_workspace_bytes(size_t n_samples, int channels, int grade, int dtype, int algo, int block_size,
                         size_t* out_bytes) {
  (void)block_size;
  if (out_bytes == nullptr) return MAVG_ERR_INVALID_ARG;
  const int st = validate(n_samples, channels, grade, dtype, algo);
  if (st != MAVG_OK) return st;
  *out_bytes = 0;
  if (n_samples == 0) return MAVG_OK;
  // the dispatch decides; ask it in plan mode (nothing is launched)
  LaunchPlan plan{};
  plan.ws_bytes = 0;
  g_plan = &plan;
  const int rs = mavg_run(reinterpret_cast<const void*>(uintptr_t(1) << 20), reinterpret_cast<void*>(uintptr_t(1) << 21),
                          n_samples, channels, grade, dtype, algo, block_size, nullptr, nullptr, 0, nullptr);
  g_plan = nullptr;
  if (rs != MAVG_OK) return rs;
  *out_bytes = plan.ws_bytes;
  return MAVG_OK;
}

int mavg_run(const void* d_in, void* d_out, size_t n_samples, int channels, int grade, int dtype, int algo,
             int block_size, const void* d_history, void* d_ws, size_t ws_bytes, void* stream) {
  (void)block_size;
  const Workspace ws{d_ws, ws_bytes};
  int st = validate(n_samples, channels, grade, dtype, algo);
  if (st != MAVG_OK) return st;
  if (n_samples == 0) return MAVG_OK;
  if (d_in == nullptr || d_out == nullptr) return MAVG_ERR_INVALID_ARG;
  algo = mavg_resolve_algo(n_samples, channels, grade, dtype, algo);
  const bool vec_possible = vec_frames(dtype, channels) > 0;
  if (is_vec_algo(algo) && vec_possible && (!aligned16(d_in) || !aligned16(d_out))) return MAVG_ERR_MISALIGNED;
  if (dtype == MAVG_I16 && !(reinterpret_cast<uintptr_t>(d_in) % 2 == 0 && reinterpret_cast<uintptr_t>(d_out) % 2 == 0))
    return MAVG_ERR_MISALIGNED;
  if (dtype == MAVG_F32 && !(reinterpret_cast<uintptr_t>(d_in) % 4 == 0 && reinterpret_cast<uintptr_t>(d_out) % 4 == 0))
    return MAVG_ERR_MISALIGNED;

  hipStream_t s = static_cast<hipStream_t>(stream);
  const long long nframes = (long long)(n_samples / (size_t)channels);
  const int C = channels;
  const int k = grade;
  const bool f32 = dtype == MAVG_F32;
  const bool i64acc = !f32 && k > 65535;

  switch (algo) {
    case MAVG_ALGO_BLELLOCH:
    case MAVG_ALGO_BLELLOCH_SCALAR:
    case MAVG_ALGO_HILLIS:
    case MAVG_ALGO_HILLIS_SCALAR: {
      const bool vec = (algo == MAVG_ALGO_BLELLOCH || algo == MAVG_ALGO_HILLIS);
      const bool hs = (algo == MAVG_ALGO_HILLIS || algo == MAVG_ALGO_HILLIS_SCALAR);
      if (f32) return scan_f32(C, vec, hs, d_in, d_out, d_history, nframes, k, s, ws);
      if (i64acc) return scan_i16_wide(C, vec, hs, d_in, d_out, d_history, nframes, k, s, ws);
      return scan_i16(C, vec, hs, d_in, d_out, d_history, nframes, k, s, ws);
    }
    case MAVG_ALGO_DIRECT:
    case MAVG_ALGO_DIRECT_VEC2:
    case MAVG_ALGO_DIRECT_SCALAR: {
      const int width = algo == MAVG_ALGO_DIRECT ? 16 : (algo == MAVG_ALGO_DIRECT_VEC2 ? 8 : 0);
      return direct_any(dtype, i64acc, C, width, d_in, d_out, d_history, nframes, k, s);
    }
    case MAVG_ALGO_NAIVE: {
      return naive_any(dtype, i64acc, d_in, d_out, d_history, nframes, C, k, s);
    }
    default: return MAVG_ERR_INVALID_ARG;
  }
}

int mavg_plan(size_t n_samples, int channels, int grade, int dtype, int algo, char* buf, size_t buflen) {
  if (buf == nullptr || buflen == 0) return MAVG_ERR_INVALID_ARG;
  buf[0] = 0;
  if (n_samples == 0) return MAVG_ERR_INVALID_ARG;
  LaunchPlan plan{};
  g_plan = &plan;
  // aligned dummy device pointers: nothing is launched or dereferenced in plan mode
  const int st = mavg_run(reinterpret_cast<const void*>(uintptr_t(1) << 20), reinterpret_cast<void*>(uintptr_t(1) << 21),
                          n_samples, channels, grade, dtype, algo, 0, nullptr, nullptr, 0, nullptr);
  g_plan = nullptr;
  if (st != MAVG_OK) return st;
  snprintf(buf, buflen, "%s", plan.text);
  return MAVG_OK;
}

int mavg_fill_synthetic(void* d_out, size_t n_samples, int dtype, uint64_t seed, uint64_t offset, int dist,
                        void* stream) {
  if (dtype != MAVG_I16 && dtype != MAVG_F32) return MAVG_ERR_INVALID_ARG;
  if (dist != 0 && dist != 1) return MAVG_ERR_INVALID_ARG;
  if (dist == 1 && dtype != MAVG_F32) return MAVG_ERR_INVALID_ARG;
  if (n_samples == 0) return MAVG_OK;
  if (d_out == nullptr) return MAVG_ERR_INVALID_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const long long n = (long long)n_samples;
  const long long want = (n + kWG - 1) / kWG;
  const unsigned grid = (unsigned)std::min<long long>(want, (long long)device_cu_count() * 16);
  if (dtype == MAVG_F32)
    hipLaunchKernelGGL(synth_kernel<float>, dim3(grid), dim3(kWG), 0, s, static_cast<float*>(d_out), n,
                       seed + offset, dist);
  else
    hipLaunchKernelGGL(synth_kernel<int16_t>, dim3(grid), dim3(kWG), 0, s, static_cast<int16_t*>(d_out), n,
                       seed + offset, dist);
  return hipGetLastError() == hipSuccess ? MAVG_OK : MAVG_ERR_HIP;
}

int mavg_stream_copy(const void* d_in, void* d_out, size_t bytes, void* stream) {
  if (bytes == 0) return MAVG_OK;
  if (d_in == nullptr || d_out == nullptr || bytes % 16 != 0) return MAVG_ERR_INVALID_ARG;
  if (!aligned16(d_in) || !aligned16(d_out)) return MAVG_ERR_MISALIGNED;
  const long long n = (long long)(bytes / 16);
  const long long grid = (n + kWG - 1) / kWG;
  if (grid > 0x7fffffffLL) return MAVG_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(stream_copy_kernel<u32x4>, dim3((unsigned)grid), dim3(kWG), 0, static_cast<hipStream_t>(stream),
                     static_cast<const u32x4*>(d_in), static_cast<u32x4*>(d_out), n);
  return hipGetLastError() == hipSuccess ? MAVG_OK : MAVG_ERR_HIP;
}

}  // extern "C"
