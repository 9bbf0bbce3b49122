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

bool aligned(const void* p, size_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; }

size_t elem_size(int dtype) { return dtype == MAVG_F32 ? 4 : 2; }

// frames per 16-B unit for (dtype, C), 0 if C*elem does not divide 16
int vec_frames(int dtype, int C) {
  const int eb = (int)elem_size(dtype);
  const int fb = eb * C;
  if (fb > 16 || 16 % fb != 0) return 0;
  return 16 / fb;
}

// Bytes of the vector unit an algorithm moves per lane access when it runs
// its vector form (16 or 8), or 0 for the frame-unit (F = 1) forms.
int vec_unit_bytes(int algo, int dtype, int C) {
  const int fb = (int)elem_size(dtype) * C;
  switch (algo) {
    case MAVG_ALGO_BLELLOCH:
    case MAVG_ALGO_HILLIS:
    case MAVG_ALGO_DIRECT: return vec_frames(dtype, C) > 0 ? 16 : 0;
    case MAVG_ALGO_DIRECT_VEC2: return (fb <= 8 && 8 % fb == 0) ? 8 : 0;
    default: return 0;
  }
}

// The frame-unit (one frame per lane) form of an algorithm family.
int scalar_form(int algo) {
  switch (algo) {
    case MAVG_ALGO_BLELLOCH: return MAVG_ALGO_BLELLOCH_SCALAR;
    case MAVG_ALGO_HILLIS: return MAVG_ALGO_HILLIS_SCALAR;
    case MAVG_ALGO_DIRECT:
    case MAVG_ALGO_DIRECT_VEC2: return MAVG_ALGO_DIRECT_SCALAR;
    default: return algo;
  }
}

int validate(size_t n, int C, int k, int dtype, int algo, int block) {
  if (dtype != MAVG_I16 && dtype != MAVG_F32) return MAVG_ERR_INVALID_ARG;
  if (algo < MAVG_ALGO_AUTO || algo > MAVG_ALGO_NAIVE) return MAVG_ERR_INVALID_ARG;
  if (C < 1 || k < 1) return MAVG_ERR_INVALID_ARG;
  if (n % (size_t)C != 0) return MAVG_ERR_INVALID_ARG;
  if (block != 0 && (block < 32 || block > 1024 || block % 32 != 0)) return MAVG_ERR_INVALID_ARG;
  if (C > kMaxChannels && algo != MAVG_ALGO_AUTO && algo != MAVG_ALGO_NAIVE) return MAVG_ERR_UNSUPPORTED;
  if (n / (size_t)C > (size_t)0x3fffffffffffffffULL) return MAVG_ERR_UNSUPPORTED;
  return MAVG_OK;
}

// k = 1: y = x / 1 = x exactly, for every algorithm and dtype (the window is
// the sample itself; no history).  A copy instead of a scan: a telescoped
// running sum loses up to ~1e-6 relative on mixed-scale fp32 data at k = 1
// (neighbours 2^30 times larger round the differences), a copy loses nothing.
// The flat non-temporal copy when both views are 16-B aligned, else hipMemcpyAsync.
int launch_identity(int dtype, int C, const Sig& sg, hipStream_t s) {
  const size_t bytes = (size_t)sg.nframes * (size_t)C * elem_size(dtype);
  const bool flat = aligned(sg.in, 16) && aligned(sg.out, 16) && bytes % 16 == 0;
  if (g_plan) {
    snprintf(g_plan->text, sizeof(g_plan->text), "copy<%s,C=%d> (k=1: y = x) bytes=%zu %s",
             dtype == MAVG_F32 ? "f32" : "i16", C, bytes, flat ? "flat nt 16-B" : "hipMemcpyAsync");
    return MAVG_OK;
  }
  if (bytes == 0) return MAVG_OK;
  if (flat) {
    const long long n = (long long)(bytes / 16);
    const long long grid = (n + kWG - 1) / kWG;
    if (grid > 0x7fffffffLL) return MAVG_ERR_UNSUPPORTED;
    hipLaunchKernelGGL(stream_copy_kernel<u32x4>, dim3((unsigned)grid), dim3(kWG), 0, s,
                       static_cast<const u32x4*>(sg.in), static_cast<u32x4*>(sg.out), n);
    return hipGetLastError() == hipSuccess ? MAVG_OK : MAVG_ERR_HIP;
  }
  return hipMemcpyAsync(sg.out, sg.in, bytes, hipMemcpyDeviceToDevice, s) == hipSuccess ? MAVG_OK : MAVG_ERR_HIP;
}

// One launch of a concrete algorithm over a view (no alignment policy here).
int launch_algo(int algo, int dtype, int C, const Sig& sg, int k, int block, hipStream_t s, Workspace ws) {
  if (k == 1) return launch_identity(dtype, C, sg, s);
  const bool f32 = dtype == MAVG_F32;
  const bool i64acc = !f32 && k > 65535;
  switch (algo) {
    case MAVG_ALGO_BLELLOCH:
    case MAVG_ALGO_BLELLOCH_SCALAR:
    case MAVG_ALGO_HILLIS:
    case MAVG_ALGO_HILLIS_SCALAR: {
      const bool vec = (algo == MAVG_ALGO_BLELLOCH || algo == MAVG_ALGO_HILLIS);
      const bool hs = (algo == MAVG_ALGO_HILLIS || algo == MAVG_ALGO_HILLIS_SCALAR);
      if (f32) return scan_f32(C, vec, hs, sg, k, block, s, ws);
      if (i64acc) return scan_i16_wide(C, vec, hs, sg, k, block, s, ws);
      return scan_i16(C, vec, hs, sg, k, block, s, ws);
    }
    case MAVG_ALGO_DIRECT:
    case MAVG_ALGO_DIRECT_VEC2:
    case MAVG_ALGO_DIRECT_SCALAR: {
      const int width = algo == MAVG_ALGO_DIRECT ? 16 : (algo == MAVG_ALGO_DIRECT_VEC2 ? 8 : 0);
      return direct_any(dtype, i64acc, C, width, sg, k, block, s);
    }
    case MAVG_ALGO_NAIVE: return naive_any(dtype, i64acc, sg, C, k, block, s);
    default: return MAVG_ERR_INVALID_ARG;
  }
}

// Workspace the launch(es) for this problem need, whatever the pointers'
// alignment: a vector algorithm on a misaligned view may run its frame-unit
// form over the whole signal instead (more, smaller look-ahead tiles).
size_t plan_ws(size_t n, int C, int k, int dtype, int algo, int block) {
  size_t need = 0;
  const int forms[2] = {algo, scalar_form(algo)};
  for (int i = 0; i < (forms[1] == forms[0] ? 1 : 2); ++i) {
    LaunchPlan plan{};
    g_plan = &plan;
    const Sig sg{reinterpret_cast<const void*>(uintptr_t(1) << 20), reinterpret_cast<void*>(uintptr_t(1) << 21),
                 nullptr, (long long)(n / (size_t)C)};
    const int st = launch_algo(forms[i], dtype, C, sg, k, block, nullptr, Workspace{});
    g_plan = nullptr;
    if (st == MAVG_OK) need = std::max(need, plan.ws_bytes);
  }
  return need;
}

}  // namespace

extern "C" {

int mavg_abi_version(void) { return MAVG_ABI_VERSION; }

const char* mavg_strerror(int status) {
  switch (status) {
    case MAVG_OK: return "ok";
    case MAVG_ERR_INVALID_ARG: return "invalid argument";
    case MAVG_ERR_UNSUPPORTED: return "unsupported configuration";
    case MAVG_ERR_MISALIGNED: return "pointer not aligned to the sample size";
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
  if (out_bytes == nullptr) return MAVG_ERR_INVALID_ARG;
  const int st = validate(n_samples, channels, grade, dtype, algo, block_size);
  if (st != MAVG_OK) return st;
  *out_bytes = 0;
  if (n_samples == 0) return MAVG_OK;
  // the dispatch decides; ask it in plan mode (nothing is launched)
  *out_bytes = plan_ws(n_samples, channels, grade, dtype,
                       mavg_resolve_algo(n_samples, channels, grade, dtype, algo), block_size);
  return MAVG_OK;
}

// Alignment policy.  A vector algorithm (16-B or 8-B lane units) needs both
// views unit-aligned.  When they are not:
//   - same offset inside a unit, a whole number of frames: the first p < F
//     frames (the "head") run in the frame-unit form of the same family, the
//     rest (the "body") in the vector form; the body's history is the head
//     itself (Sig::pre) followed, further back, by the caller's history;
//   - otherwise the frame-unit form runs over the whole signal.
// A frame-unit launch whose frames are not aligned to their own (vector)
// size moves them as element accesses (Sig::eio).  Results are identical in
// every case; only element alignment is required.
int mavg_run(const void* d_in, void* d_out, size_t n_samples, int channels, int grade, int dtype, int algo,
             int block_size, const void* d_history, void* d_ws, size_t ws_bytes, void* stream) {
  const Workspace ws{d_ws, ws_bytes};
  int st = validate(n_samples, channels, grade, dtype, algo, block_size);
  if (st != MAVG_OK) return st;
  if (n_samples == 0) return MAVG_OK;
  if (d_in == nullptr || d_out == nullptr) return MAVG_ERR_INVALID_ARG;
  const size_t eb = elem_size(dtype);
  if (!aligned(d_in, eb) || !aligned(d_out, eb) || (d_history != nullptr && !aligned(d_history, eb)))
    return MAVG_ERR_MISALIGNED;
  algo = mavg_resolve_algo(n_samples, channels, grade, dtype, algo);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int C = channels;
  const size_t fb = eb * (size_t)C;
  const long long nframes = (long long)(n_samples / (size_t)C);
  // frame-unit launches: element IO when a frame is not aligned to its own vector size
  auto frame_sig = [&](const void* in, void* out, const void* hist, long long nf, int pre) {
    Sig sg{in, out, hist, nf, pre, 0};
    const bool pow2 = (fb & (fb - 1)) == 0 && fb <= 32;
    if (pow2 && (!aligned(in, fb) || !aligned(out, fb))) sg.eio = 1;
    return sg;
  };
  const int vu = vec_unit_bytes(algo, dtype, C);
  if (vu == 0) return launch_algo(algo, dtype, C, frame_sig(d_in, d_out, d_history, nframes, 0), grade, block_size, s, ws);
  if (aligned(d_in, vu) && aligned(d_out, vu))
    return launch_algo(algo, dtype, C, Sig{d_in, d_out, d_history, nframes}, grade, block_size, s, ws);
  const size_t ai = reinterpret_cast<uintptr_t>(d_in) % (size_t)vu;
  const size_t ao = reinterpret_cast<uintptr_t>(d_out) % (size_t)vu;
  const int sf = scalar_form(algo);
  if (ai != ao || ai % fb != 0)
    return launch_algo(sf, dtype, C, frame_sig(d_in, d_out, d_history, nframes, 0), grade, block_size, s, ws);
  const long long p = std::min<long long>(nframes, (long long)(((size_t)vu - ai) / fb));
  const Sig head = frame_sig(d_in, d_out, d_history, p, 0);
  const size_t off = (size_t)p * fb;
  const void* hist_body = d_history != nullptr ? static_cast<const char*>(d_history) + off : nullptr;
  const Sig body{static_cast<const char*>(d_in) + off, static_cast<char*>(d_out) + off, hist_body, nframes - p,
                 (int)p, 0};
  // both launches are first made in plan mode: an error of the second one
  // (e.g. a workspace that covers the head but not the body) must leave
  // nothing on the stream (mavg.h)
  for (int part = 0; part < (p == nframes ? 1 : 2); ++part) {
    LaunchPlan plan{};
    g_plan = &plan;
    st = part == 0 ? launch_algo(sf, dtype, C, head, grade, block_size, nullptr, ws)
                   : launch_algo(algo, dtype, C, body, grade, block_size, nullptr, ws);
    g_plan = nullptr;
    if (st != MAVG_OK) return st;
    if (plan.ws_bytes > 0 && (d_ws == nullptr || ws_bytes < plan.ws_bytes)) return MAVG_ERR_WORKSPACE;
    if (plan.ws_bytes > 0 && !aligned(d_ws, 16)) return MAVG_ERR_MISALIGNED;
  }
  st = launch_algo(sf, dtype, C, head, grade, block_size, s, ws);
  if (st != MAVG_OK || p == nframes) return st;
  return launch_algo(algo, dtype, C, body, grade, block_size, s, ws);
}

int mavg_plan(size_t n_samples, int channels, int grade, int dtype, int algo, int block_size, char* buf,
              size_t buflen) {
  if (buf == nullptr || buflen == 0) return MAVG_ERR_INVALID_ARG;
  buf[0] = 0;
  if (n_samples == 0) return MAVG_ERR_INVALID_ARG;
  const int st0 = validate(n_samples, channels, grade, dtype, algo, block_size);
  if (st0 != MAVG_OK) return st0;
  LaunchPlan plan{};
  g_plan = &plan;
  // 16-B-aligned dummy device pointers: nothing is launched or dereferenced in plan mode
  const Sig sg{reinterpret_cast<const void*>(uintptr_t(1) << 20), reinterpret_cast<void*>(uintptr_t(1) << 21),
               nullptr, (long long)(n_samples / (size_t)channels)};
  const int st = launch_algo(mavg_resolve_algo(n_samples, channels, grade, dtype, algo), dtype, channels, sg, grade,
                             block_size, nullptr, Workspace{});
  g_plan = nullptr;
  if (st != MAVG_OK) return st;
  snprintf(buf, buflen, "%s", plan.text);
  return MAVG_OK;
}

int mavg_fill_synthetic(void* d_out, size_t n_samples, int dtype, uint64_t seed, uint64_t offset, int dist,
                        void* stream) {
  if (dtype != MAVG_I16 && dtype != MAVG_F32) return MAVG_ERR_INVALID_ARG;
  if (dist < 0 || dist > 2) return MAVG_ERR_INVALID_ARG;
  if (dist != 0 && dtype != MAVG_F32) return MAVG_ERR_INVALID_ARG;
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
  if (!aligned(d_in, 16) || !aligned(d_out, 16)) return MAVG_ERR_MISALIGNED;
  const long long n = (long long)(bytes / 16);
  const long long grid = (n + kWG - 1) / kWG;
  if (grid > 0x7fffffffLL) return MAVG_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(stream_copy_kernel<u32x4>, dim3((unsigned)grid), dim3(kWG), 0, static_cast<hipStream_t>(stream),
                     static_cast<const u32x4*>(d_in), static_cast<u32x4*>(d_out), n);
  return hipGetLastError() == hipSuccess ? MAVG_OK : MAVG_ERR_HIP;
}

}  // extern "C"
