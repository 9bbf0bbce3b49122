// host_utils.hpp -- host-side infrastructure of the bin_* CLIs, written for
// HIP on MI355X.  Behavioural counterpart of the reference's gpu_utils.h and
// benchmark.h: the same timing model (warm-up 5 + 10 measured rounds,
// gpu_utils.h:31-32), the same stdout report (ProfileResult::print_stats,
// benchmark.h:33-69) and the same CSV schema (CsvLogger, gpu_utils.h:162-231),
// so the harness and any downstream CSV tooling see identical output.
// Differences by design: HIP_CHECK reports and returns instead of exit()ing
// from library code, kernels are launched through libmavg's C ABI, and the
// workspace holds no halo zone (the ABI takes an explicit history pointer).
#pragma once

#include <hip/hip_runtime.h>
#include <sys/stat.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <stdexcept>
#include <string>

#include "../../include/mavg.h"

namespace mavg_cli {

// CLI-level check: a failed HIP call ends the program with a non-zero status
// (the reference exits with EXIT_FAILURE too, gpu_utils.h:10-18).
#define HIP_CHECK(call)                                                                              \
  do {                                                                                               \
    hipError_t err_ = (call);                                                                        \
    if (err_ != hipSuccess) {                                                                        \
      std::fprintf(stderr, "HIP Error: %s at %s:%d\n", hipGetErrorString(err_), __FILE__, __LINE__); \
      std::exit(EXIT_FAILURE);                                                                       \
    }                                                                                                \
  } while (0)

#define MAVG_CHECK(call)                                                                                   \
  do {                                                                                                     \
    int st_ = (call);                                                                                      \
    if (st_ != MAVG_OK) {                                                                                  \
      std::fprintf(stderr, "libmavg error: %s (status %d) at %s:%d\n", mavg_strerror(st_), st_, __FILE__, \
                   __LINE__);                                                                              \
      std::exit(EXIT_FAILURE);                                                                             \
    }                                                                                                      \
  } while (0)

constexpr int warmupRounds = 5;
constexpr int measurementRounds = 10;

enum class MemoryMode { Standard, Unified };

template <MemoryMode Mode> struct MemoryTraits;

template <> struct MemoryTraits<MemoryMode::Standard> {
  static const char* name() { return "Standard"; }
  static void allocate(void** p, size_t bytes) { HIP_CHECK(hipMalloc(p, bytes)); }
  static void release(void* p) { (void)hipFree(p); }
  static void copyH2D(void* dst, const void* src, size_t bytes) {
    HIP_CHECK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
  }
  static void copyD2H(void* dst, const void* src, size_t bytes) {
    HIP_CHECK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  }
};

// Managed memory (the reference's zero-copy mode, gpu_utils.h MemoryTraits):
// the host writes the input in place and the kernel reads it where it lies.
// Prefetching the pages to the GPU inside the H2D phase was measured
// (profiles/r02_cli_unified_prefetch/): the kernel phase then drops from 2.59
// to 0.042 ms on 50 M samples, but the migration takes 149 ms (H2D) + 30 ms
// (D2H) on this driver (no XNACK), 19x the zero-copy form's 9.3 ms end to
// end -- so the zero-copy form stays, and its Compute column includes the
// link traffic by construction.
template <> struct MemoryTraits<MemoryMode::Unified> {
  static const char* name() { return "Unified"; }
  static void allocate(void** p, size_t bytes) { HIP_CHECK(hipMallocManaged(p, bytes)); }
  static void release(void* p) { (void)hipFree(p); }
  static void copyH2D(void* dst, const void* src, size_t bytes) { std::memcpy(dst, src, bytes); }
  static void copyD2H(void* dst, const void* src, size_t bytes) {
    HIP_CHECK(hipDeviceSynchronize());
    std::memcpy(dst, src, bytes);
  }
};

// Device buffers for one run: input, output and libmavg's workspace.
template <typename T, MemoryMode Mode>
class DspWorkspace {
 public:
  T* input = nullptr;
  T* output = nullptr;
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  const size_t count;

  DspWorkspace(size_t n, size_t ws_bytes) : scratch_bytes(ws_bytes), count(n) {
    const size_t bytes = (n ? n : 1) * sizeof(T);
    MemoryTraits<Mode>::allocate(reinterpret_cast<void**>(&input), bytes);
    MemoryTraits<Mode>::allocate(reinterpret_cast<void**>(&output), bytes);
    if (scratch_bytes) {
      MemoryTraits<Mode>::allocate(&scratch, scratch_bytes);
      HIP_CHECK(hipMemset(scratch, 0, scratch_bytes));
    }
  }
  ~DspWorkspace() {
    MemoryTraits<Mode>::release(input);
    MemoryTraits<Mode>::release(output);
    if (scratch) MemoryTraits<Mode>::release(scratch);
  }
  DspWorkspace(const DspWorkspace&) = delete;
  DspWorkspace& operator=(const DspWorkspace&) = delete;
};

// Phases of one timed iteration (benchmark.h:9-31); print_stats reproduces
// the reference's report line for line (benchmark.h:33-69).
struct ProfileResult {
  float initialization_ms = 0.0f;
  float transfer_h2d_ms = 0.0f;
  float compute_ms = 0.0f;
  float transfer_d2h_ms = 0.0f;
  float total_ms = 0.0f;

  void operator+=(const ProfileResult& o) {
    initialization_ms += o.initialization_ms;
    transfer_h2d_ms += o.transfer_h2d_ms;
    compute_ms += o.compute_ms;
    transfer_d2h_ms += o.transfer_d2h_ms;
    total_ms += o.total_ms;
  }
  void divide(int k) {
    if (k == 0) return;
    initialization_ms /= k;
    transfer_h2d_ms /= k;
    compute_ms /= k;
    transfer_d2h_ms /= k;
    total_ms /= k;
  }
  void print_stats(size_t n, size_t in_size, size_t out_size = 0) const {
    if (out_size == 0) out_size = in_size;
    const double gb = (double)n * (double)(in_size + out_size) / 1e9;
    const double ms_samples = (double)n / 1e6;
    const double kernel_sec = compute_ms / 1000.0;
    const double total_sec = total_ms / 1000.0;
    const double cold_sec = (initialization_ms + total_ms) / 1000.0;
    std::cout << std::fixed << std::setprecision(3);
    std::cout << "1. LATENCY BREAKDOWN (Steady State)" << std::endl;
    if (transfer_h2d_ms > 0) std::cout << "   H2D Transfer:   " << transfer_h2d_ms << " ms" << std::endl;
    std::cout << "   Kernel Compute: " << compute_ms << " ms" << std::endl;
    if (transfer_d2h_ms > 0) std::cout << "   D2H Transfer:   " << transfer_d2h_ms << " ms" << std::endl;
    std::cout << "   -----------------------------" << std::endl;
    std::cout << "   TOTAL LATENCY:  " << total_ms << " ms" << std::endl;
    std::cout << "\n2. THROUGHPUT (Steady State)" << std::endl;
    if (compute_ms > 0) {
      std::cout << "   Kernel Bandwidth: " << (gb / kernel_sec) << " GB/s" << std::endl;
      std::cout << "   Kernel Speed:   " << (ms_samples / kernel_sec) << " Mega Samples/s" << std::endl;
    }
    std::cout << "   App BandWidth:   " << (gb / total_sec) << " GB/s" << std::endl;
    std::cout << "   App Speed:      " << (ms_samples / total_sec) << " Mega Samples/s" << std::endl;
    std::cout << "   Cold Start:     " << (ms_samples / cold_sec) << " Mega Samples/s (Includes Init)" << std::endl;
    std::cout << "\n3. INITIALIZATION COST (One-time)" << std::endl;
    std::cout << "   Allocation:     " << initialization_ms << " ms" << std::endl;
    std::cout << "   First Frame:    " << (initialization_ms + total_ms) << " ms (Cold Start)" << std::endl;
    std::cout << "___________________________________\n" << std::endl;
  }
};

// start -> h2d -> compute -> stop on hipEvents (benchmark.h:72-96); the
// events are recorded on the stream the work is enqueued on.
class GpuTimer {
  hipEvent_t start_evt{}, h2d_evt{}, compute_evt{}, stop_evt{};
  hipStream_t stream_;

 public:
  explicit GpuTimer(hipStream_t s = nullptr) : stream_(s) {
    HIP_CHECK(hipEventCreate(&start_evt));
    HIP_CHECK(hipEventCreate(&h2d_evt));
    HIP_CHECK(hipEventCreate(&compute_evt));
    HIP_CHECK(hipEventCreate(&stop_evt));
  }
  ~GpuTimer() {
    (void)hipEventDestroy(start_evt);
    (void)hipEventDestroy(h2d_evt);
    (void)hipEventDestroy(compute_evt);
    (void)hipEventDestroy(stop_evt);
  }
  hipStream_t stream() const { return stream_; }
  void start() { HIP_CHECK(hipEventRecord(start_evt, stream_)); }
  void mark_h2d() { HIP_CHECK(hipEventRecord(h2d_evt, stream_)); }
  void mark_compute() { HIP_CHECK(hipEventRecord(compute_evt, stream_)); }
  void stop() {
    HIP_CHECK(hipEventRecord(stop_evt, stream_));
    HIP_CHECK(hipEventSynchronize(stop_evt));
  }
  ProfileResult get_result() {
    ProfileResult r;
    HIP_CHECK(hipEventElapsedTime(&r.transfer_h2d_ms, start_evt, h2d_evt));
    HIP_CHECK(hipEventElapsedTime(&r.compute_ms, h2d_evt, compute_evt));
    HIP_CHECK(hipEventElapsedTime(&r.transfer_d2h_ms, compute_evt, stop_evt));
    r.total_ms = r.transfer_h2d_ms + r.compute_ms + r.transfer_d2h_ms;
    return r;
  }
};

class CpuTimer {
  using Clock = std::chrono::high_resolution_clock;
  std::chrono::time_point<Clock> t_start, t_end;

 public:
  void start() { t_start = Clock::now(); }
  void mark_h2d() {}
  void mark_compute() {}
  void stop() { t_end = Clock::now(); }
  ProfileResult get_result() {
    ProfileResult r;
    const auto us = std::chrono::duration_cast<std::chrono::microseconds>(t_end - t_start);
    r.compute_ms = us.count() / 1000.0f;
    r.total_ms = r.compute_ms;
    return r;
  }
};

// warm-up, then average `iterations` measured runs (benchmark.h:116-132)
template <typename TimerType, typename Func>
ProfileResult benchmark(TimerType& timer, int iterations, int warmup, Func body) {
  for (int i = 0; i < warmup; ++i) body(timer);
  ProfileResult avg;
  for (int i = 0; i < iterations; ++i) {
    body(timer);
    avg += timer.get_result();
  }
  avg.divide(iterations);
  return avg;
}

// Appends one row per run to a CSV with the reference's 14-column schema
// (gpu_utils.h:196-199); header written when the file is new.
class CsvLogger {
  std::string filename;
  static bool exists(const std::string& f) {
    struct stat b;
    return stat(f.c_str(), &b) == 0;
  }

 public:
  explicit CsvLogger(std::string f = "benchmark_data.csv") : filename(std::move(f)) {}
  void log(const std::string& algo, const std::string& mode, size_t N, int grade, int block,
           const ProfileResult& r, size_t in_bytes, size_t out_bytes = 0) {
    if (out_bytes == 0) out_bytes = in_bytes;
    const bool fresh = !exists(filename);
    std::ofstream f(filename, std::ios::app);
    if (!f.is_open()) {
      std::cerr << "Error: Could not open CSV file " << filename << std::endl;
      return;
    }
    if (fresh)
      f << "Algorithm,MemoryMode,N_Samples,Grade,BlockSize,"
        << "H2D_ms,Compute_ms,D2H_ms,Total_ms,"
        << "Init_ms,ColdStart_Total_ms,"
        << "Bandwidth_GBs,Throughput_MSs,ColdStart_MSs\n";
    const double gb = (double)N * (double)(in_bytes + out_bytes) / 1e9;
    const double ms = (double)N / 1e6;
    const double steady = r.total_ms / 1000.0;
    const double cold = (r.initialization_ms + r.total_ms) / 1000.0;
    f << algo << "," << mode << "," << N << "," << grade << "," << block << "," << r.transfer_h2d_ms << ","
      << r.compute_ms << "," << r.transfer_d2h_ms << "," << r.total_ms << "," << r.initialization_ms << ","
      << (r.initialization_ms + r.total_ms) << "," << (steady > 0 ? gb / steady : 0.0) << ","
      << (steady > 0 ? ms / steady : 0.0) << "," << (cold > 0 ? ms / cold : 0.0) << "\n";
    std::cout << ">> Data saved to " << filename << std::endl;
  }
};

}  // namespace mavg_cli
