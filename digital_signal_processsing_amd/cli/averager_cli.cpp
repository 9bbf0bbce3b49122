// averager_cli.cpp -- the per-variant command-line programs (bin_cpu,
// bin_parallel, bin_shared, bin_vec2, bin_vec4, bin_hillis, bin_vhillis,
// bin_blelloch, bin_vblelloch), compiled once per variant with
// -DMAVG_VARIANT=<index into kVariants>.
//
// Drop-in for the reference binaries (README.md:34-42, run_benchmarks.py:8-18):
//   argv      <wav_path> <grade> <block_size>; usage error -> exit 1 when
//             argc < 4 or block_size is not a multiple of 32 in [32, 1024]
//             (e.g. blelloch_scan_averager.cu:313-327)
//   stdout    banner + "MEM MODE" sections + ProfileResult::print_stats
//   CSV       two rows per GPU binary (Standard, Unified), one for bin_cpu
//             (RAM, block 0) appended to ./benchmark_data.csv
// Deliberate differences: a WAV read failure exits 1 (the
// reference exits 0); grade < 1 is rejected (the reference divides by zero);
// the int16 results are bit-exact with the serial reference on every variant
// (the reference's GPU variants round through a float reciprocal); the scan
// variants move int16 over PCIe (the reference widens to int64 on the host),
// so their CSV bandwidth is computed on 2 B in + 2 B out per sample.
// Optional trailing flags: --out <wav> (write the filtered signal),
// --modes standard|unified|both, --csv <file>.
// Synthetic north-star mode (BASELINE.json configs):
//   bin_<variant> - <grade> <block> --synthetic <n_samples> [--dtype f32|i16]
//                 [--channels C] [--seed S] [--verify]
// replaces the WAV with the counter-based signal generated in place on the
// device (mavg_fill_synthetic; bin_cpu generates the same values on the
// host), so the timed region is the kernel on HBM-resident data: no H2D/D2H.
// It prints the report plus a roofline section (algorithmic bytes: one read
// and one write per sample, against 8 TB/s) and logs one CSV row with
// MemoryMode "Device".  --verify checks sampled output spans against a
// direct window sum of the regenerated input (int16 bit-exact, fp32 within
// 1e-5 relative); --out <file> writes the raw output samples (native-endian
// T, no header) instead of a WAV.
#include <algorithm>
#include <cstdint>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <iomanip>
#include <iostream>
#include <string>
#include <vector>

#include "host_utils.hpp"
#include "wav_io.hpp"

using namespace mavg_cli;

namespace {

struct Variant {
  const char* bin;
  const char* csv_name;  // Algorithm column, as the reference logs it
  int algo;              // mavg_algo; -1 = the CPU variant
  const char* banner;    // nullptr: the reference variant prints none
};

// index = MAVG_VARIANT; csv names from the reference's logger.log() calls
constexpr Variant kVariants[] = {
    {"bin_cpu", "SingleThreadCpu", -1, "--- Single Thread Averager ---"},
    {"bin_parallel", "Parallel Averager", MAVG_ALGO_NAIVE, "--- SIMPLE PARALLEL AVERAGER ---"},
    {"bin_shared", "SM Parallel Averager", MAVG_ALGO_DIRECT_SCALAR, "--- SHARED MEMORY PARALLEL AVERAGER ---"},
    {"bin_vec2", "Vectorized SM Parallel Averager", MAVG_ALGO_DIRECT_VEC2, nullptr},
    {"bin_vec4", "Vectorized SM4 Parallel", MAVG_ALGO_DIRECT, nullptr},
    {"bin_hillis", "HillisSteele", MAVG_ALGO_HILLIS_SCALAR, "--- Hillis Steele Averager ---"},
    {"bin_vhillis", "Vectorized HillisSteele", MAVG_ALGO_HILLIS, nullptr},
    {"bin_blelloch", "Blelloch", MAVG_ALGO_BLELLOCH_SCALAR, nullptr},
    {"bin_vblelloch", "Vectorized Blelloch", MAVG_ALGO_BLELLOCH, nullptr},
};

#ifndef MAVG_VARIANT
#error "compile with -DMAVG_VARIANT=<0..8>"
#endif
constexpr Variant kV = kVariants[MAVG_VARIANT];

struct Options {
  std::string wav, out, csv = "benchmark_data.csv";
  int grade = 0, block = 0;
  bool standard = true, unified = true;
  // synthetic mode
  size_t synth_n = 0;  // 0: WAV mode
  int dtype = MAVG_F32, channels = 1;
  uint64_t seed = 0x5EED;
  bool verify = false;
};

constexpr double kHbmPeakGBs = 8000.0;  // MI355X HBM3E spec peak

// the device generator's value for global sample i (mavg_fill_synthetic,
// dist 0): int16-valued, as int16 or as float
uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
template <typename T> T synth_value(uint64_t seed, size_t i) {
  return (T)(int16_t)(uint16_t)(splitmix64(seed + (uint64_t)i) >> 48);
}

// The product's own single-thread CPU averager (bin_cpu): the serial
// running-sum loop of profilable_moving_averager.cpp:14-37 with the
// warm-up clamped to the frame count.
void cpu_averager(int C, int k, const std::vector<int16_t>& x, std::vector<int16_t>& y) {
  const size_t frames = x.size() / (size_t)C;
  std::vector<int64_t> sum((size_t)C, 0);
  const size_t warm = std::min((size_t)k, frames);
  for (size_t i = 0; i < warm; ++i)
    for (int c = 0; c < C; ++c) {
      sum[c] += x[i * C + c];
      y[i * C + c] = (int16_t)(sum[c] / k);
    }
  for (size_t i = (size_t)k; i < frames; ++i)
    for (int c = 0; c < C; ++c) {
      sum[c] += x[i * C + c] - x[(i - k) * C + c];
      y[i * C + c] = (int16_t)(sum[c] / k);
    }
}

// fp32 counterpart: the same loop with an fp64 running sum,
// output fl32(sum / k)
void cpu_averager(int C, int k, const std::vector<float>& x, std::vector<float>& y) {
  const size_t frames = x.size() / (size_t)C;
  std::vector<double> sum((size_t)C, 0.0);
  const size_t warm = std::min((size_t)k, frames);
  for (size_t i = 0; i < warm; ++i)
    for (int c = 0; c < C; ++c) {
      sum[c] += x[i * C + c];
      y[i * C + c] = (float)(sum[c] / k);
    }
  for (size_t i = (size_t)k; i < frames; ++i)
    for (int c = 0; c < C; ++c) {
      sum[c] += (double)x[i * C + c] - (double)x[(i - k) * C + c];
      y[i * C + c] = (float)(sum[c] / k);
    }
}

int run_cpu(const Options& o, int C, const std::vector<int16_t>& samples, std::vector<int16_t>& out) {
  CsvLogger logger(o.csv);
  std::cout << kV.banner << std::endl;
  std::cout << "total samples: " << samples.size() << std::endl;
  std::cout << "point: " << o.grade << std::endl;
  CpuTimer timer;
  ProfileResult init = benchmark(timer, 25, 5, [&](CpuTimer& t) {
    t.start();
    std::vector<int16_t> tmp(samples.size());
    t.stop();
  });
  ProfileResult res = benchmark(timer, measurementRounds, warmupRounds, [&](CpuTimer& t) {
    t.start();
    cpu_averager(C, o.grade, samples, out);
    t.stop();
  });
  res.initialization_ms = init.compute_ms;
  res.print_stats(samples.size(), sizeof(int16_t));
  logger.log(kV.csv_name, "RAM", samples.size(), o.grade, 0, res, sizeof(int16_t));
  return 0;
}

// one timed iteration: H2D -> libmavg kernel -> D2H (blellochAveragerGpuLoad,
// blelloch_scan_averager.cu:189-232, and its siblings)
template <MemoryMode Mode>
void gpu_load(DspWorkspace<int16_t, Mode>& ws, const Options& o, int C, size_t n, GpuTimer& t,
              const std::vector<int16_t>& samples, std::vector<int16_t>& out) {
  t.start();
  MemoryTraits<Mode>::copyH2D(ws.input, samples.data(), n * sizeof(int16_t));
  t.mark_h2d();
  MAVG_CHECK(mavg_run(ws.input, ws.output, n, C, o.grade, MAVG_I16, kV.algo, o.block, nullptr, ws.scratch,
                      ws.scratch_bytes, t.stream()));
  t.mark_compute();
  MemoryTraits<Mode>::copyD2H(out.data(), ws.output, n * sizeof(int16_t));
  t.stop();
}

template <MemoryMode Mode>
void profile_mode(const Options& o, int C, size_t n, const std::vector<int16_t>& samples,
                  std::vector<int16_t>& out, CsvLogger& logger) {
  size_t ws_bytes = 0;
  MAVG_CHECK(mavg_workspace_bytes(n, C, o.grade, MAVG_I16, kV.algo, o.block, &ws_bytes));
  CpuTimer ct;
  ProfileResult init = benchmark(ct, measurementRounds, warmupRounds, [&](CpuTimer& t) {
    t.start();
    DspWorkspace<int16_t, Mode> tmp(n, ws_bytes);
    t.stop();
  });
  DspWorkspace<int16_t, Mode> ws(n, ws_bytes);
  GpuTimer gt(nullptr);
  ProfileResult res = benchmark(gt, measurementRounds, warmupRounds, [&](GpuTimer& t) {
    gpu_load<Mode>(ws, o, C, n, t, samples, out);
  });
  res.initialization_ms = init.compute_ms;
  res.print_stats(samples.size(), sizeof(int16_t));
  logger.log(kV.csv_name, MemoryTraits<Mode>::name(), samples.size(), o.grade, o.block, res, sizeof(int16_t));
}

int run_gpu(const Options& o, int C, const std::vector<int16_t>& samples, std::vector<int16_t>& out) {
  CsvLogger logger(o.csv);
  const size_t n = samples.size() / (size_t)C * (size_t)C;  // whole frames
  if (kV.banner) {  // the variant's own header (hillis_steele_averager.cu:205-207, profilable_*.cu)
    std::cout << kV.banner << std::endl;
    if (kV.algo == MAVG_ALGO_HILLIS_SCALAR) {
      std::cout << "total samples: " << samples.size() << std::endl;
      std::cout << "point: " << o.grade << std::endl;
    } else {
      std::cout << "Samples: " << samples.size() << std::endl;
      std::cout << "point: " << o.grade << std::endl;
      std::cout << "block Size: " << o.block << std::endl;
    }
  }
  {  // the launch the block size maps to (workgroup = the next power of two >= 64,
     // see mavg.h): on stderr, so stdout stays the reference's report
    char plan[512] = {0};
    if (n > 0) MAVG_CHECK(mavg_plan(n, C, o.grade, MAVG_I16, kV.algo, o.block, plan, sizeof(plan)));
    std::cerr << "Kernel: " << plan << std::endl;
  }
  if (o.standard) {
    std::cout << "\n--- MEM MODE: STANDARD (Discrete) ---" << std::endl;
    profile_mode<MemoryMode::Standard>(o, C, n, samples, out, logger);
  }
  if (o.unified) {
    std::cout << "\n--- MODE: UNIFIED (Zero-Copy) ---" << std::endl;
    profile_mode<MemoryMode::Unified>(o, C, n, samples, out, logger);
  }
  return 0;
}

// ---- synthetic mode --------------------------------------------------------

const char* dtype_name(int dt) { return dt == MAVG_F32 ? "f32" : "i16"; }

void print_roofline(size_t n, size_t elem, float kernel_ms, float median_ms) {
  const double alg = 2.0 * (double)elem * (double)n;
  const double gbs = alg / (kernel_ms * 1e-3) / 1e9;
  std::cout << std::fixed << std::setprecision(3);
  std::cout << "4. ROOFLINE (HBM-resident synthetic input)" << std::endl;
  std::cout << "   Kernel median:  " << median_ms << " ms" << std::endl;
  std::cout << "   Gsamples/s:     " << (double)n / (kernel_ms * 1e-3) / 1e9 << std::endl;
  std::cout << "   HBM GB/s:       " << gbs << " (algorithmic " << 2 * elem << " B/sample)" << std::endl;
  std::cout << "   of 8 TB/s peak: " << gbs / kHbmPeakGBs << std::endl;
  std::cout << "___________________________________\n" << std::endl;
}

// direct window sums of the regenerated input over sampled output spans
template <typename T>
int verify_spans(const Options& o, size_t frames, const T* d_out) {
  const int C = o.channels, k = o.grade;
  std::vector<std::pair<size_t, size_t>> spans;  // [f0, f1)
  spans.push_back({0, std::min<size_t>(frames, 4096)});
  uint64_t r = o.seed ^ 0xC0FFEEull;
  for (int i = 0; i < 16 && frames > 256; ++i) {
    r = splitmix64(r);
    const size_t f0 = (size_t)(r % (frames - 255));
    spans.push_back({f0, f0 + 256});
  }
  if (frames > 256) spans.push_back({frames - 256, frames});
  size_t bad = 0, checked = 0;
  double worst = 0.0;
  for (auto [f0, f1] : spans) {
    std::vector<T> got((f1 - f0) * C);
    HIP_CHECK(hipMemcpy(got.data(), d_out + f0 * C, got.size() * sizeof(T), hipMemcpyDeviceToHost));
    for (int c = 0; c < C; ++c) {
      // window sum ending at frame f0, then slide (exact: int64 / fp64 of int16 values)
      int64_t s = 0;
      for (long long j = (long long)f0 - k + 1; j <= (long long)f0; ++j)
        if (j >= 0) s += (int64_t)synth_value<T>(o.seed, (size_t)j * C + c);
      for (size_t f = f0; f < f1; ++f) {
        if (f > f0) {
          s += (int64_t)synth_value<T>(o.seed, f * C + c);
          if ((long long)f - k >= 0) s -= (int64_t)synth_value<T>(o.seed, (f - k) * C + c);
        }
        const T y = got[(f - f0) * C + c];
        bool ok;
        if constexpr (sizeof(T) == 2) {
          ok = y == (T)(s / k);
        } else {
          const double e = (double)(float)((double)s / k);
          const double err = std::fabs((double)y - e) / std::max(1e-30, std::fabs(e));
          worst = std::max(worst, err);
          ok = err <= 1e-5;
        }
        bad += !ok;
        ++checked;
      }
    }
  }
  std::cout << "VERIFY: " << checked << " outputs in " << spans.size() << " spans, " << bad << " mismatches";
  if (sizeof(T) == 4) std::cout << ", max rel err " << std::scientific << worst << std::fixed;
  std::cout << std::endl;
  return bad == 0 ? 0 : 2;
}

template <typename T>
bool write_raw(const std::string& path, const T* data, size_t n) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (f == nullptr) return false;
  const bool ok = std::fwrite(data, sizeof(T), n, f) == n;
  return std::fclose(f) == 0 && ok;
}

template <typename T>
int run_gpu_synthetic(const Options& o) {
  const int C = o.channels;
  const size_t n = o.synth_n / (size_t)C * (size_t)C;
  CsvLogger logger(o.csv);
  char plan[512] = {0};
  MAVG_CHECK(mavg_plan(n, C, o.grade, o.dtype, kV.algo, o.block, plan, sizeof(plan)));
  std::cout << "--- SYNTHETIC " << dtype_name(o.dtype) << " (" << kV.csv_name << ") ---" << std::endl;
  std::cout << "Samples: " << n << "  channels: " << C << "  point: " << o.grade << "  block Size: " << o.block
            << std::endl;
  std::cout << "Kernel: " << plan << std::endl;
  size_t ws_bytes = 0;
  MAVG_CHECK(mavg_workspace_bytes(n, C, o.grade, o.dtype, kV.algo, o.block, &ws_bytes));
  CpuTimer ct;
  ct.start();
  T *d_in = nullptr, *d_out = nullptr;
  void* d_ws = nullptr;
  HIP_CHECK(hipMalloc(&d_in, std::max<size_t>(n, 1) * sizeof(T)));
  HIP_CHECK(hipMalloc(&d_out, std::max<size_t>(n, 1) * sizeof(T)));
  if (ws_bytes) HIP_CHECK(hipMalloc(&d_ws, ws_bytes));
  ct.stop();
  MAVG_CHECK(mavg_fill_synthetic(d_in, n, o.dtype, o.seed, 0, 0, nullptr));
  HIP_CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  HIP_CHECK(hipEventCreate(&e0));
  HIP_CHECK(hipEventCreate(&e1));
  auto launch = [&]() {
    MAVG_CHECK(mavg_run(d_in, d_out, n, C, o.grade, o.dtype, kV.algo, o.block, nullptr, d_ws, ws_bytes, nullptr));
  };
  for (int i = 0; i < warmupRounds; ++i) launch();
  std::vector<float> ms;
  for (int i = 0; i < measurementRounds; ++i) {
    HIP_CHECK(hipEventRecord(e0, nullptr));
    launch();
    HIP_CHECK(hipEventRecord(e1, nullptr));
    HIP_CHECK(hipEventSynchronize(e1));
    float t = 0.f;
    HIP_CHECK(hipEventElapsedTime(&t, e0, e1));
    ms.push_back(t);
  }
  ProfileResult res;
  for (float t : ms) res.compute_ms += t;
  res.compute_ms /= (float)ms.size();
  res.total_ms = res.compute_ms;
  res.initialization_ms = ct.get_result().compute_ms;
  std::vector<float> sorted = ms;
  std::sort(sorted.begin(), sorted.end());
  std::cout << "\n--- MEM MODE: DEVICE (HBM-resident, synthetic) ---" << std::endl;
  res.print_stats(n, sizeof(T));
  print_roofline(n, sizeof(T), res.compute_ms, sorted[sorted.size() / 2]);
  logger.log(kV.csv_name, "Device", n, o.grade, o.block, res, sizeof(T));
  int rc = 0;
  if (o.verify) rc = verify_spans<T>(o, n / C, d_out);
  if (rc == 0 && !o.out.empty()) {
    std::vector<T> y(n);
    HIP_CHECK(hipMemcpy(y.data(), d_out, n * sizeof(T), hipMemcpyDeviceToHost));
    if (!write_raw(o.out, y.data(), n)) {
      std::cerr << "Error: could not write " << o.out << std::endl;
      rc = 1;
    }
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(d_in);
  (void)hipFree(d_out);
  if (d_ws) (void)hipFree(d_ws);
  return rc;
}

template <typename T>
int run_cpu_synthetic(const Options& o) {
  const int C = o.channels;
  const size_t n = o.synth_n / (size_t)C * (size_t)C;
  CsvLogger logger(o.csv);
  std::cout << kV.banner << " (synthetic " << dtype_name(o.dtype) << ")" << std::endl;
  std::cout << "total samples: " << n << std::endl;
  std::cout << "point: " << o.grade << std::endl;
  std::vector<T> x(n), y(n);
  for (size_t i = 0; i < n; ++i) x[i] = synth_value<T>(o.seed, i);
  CpuTimer timer;
  ProfileResult res = benchmark(timer, measurementRounds, warmupRounds, [&](CpuTimer& t) {
    t.start();
    cpu_averager(C, o.grade, x, y);
    t.stop();
  });
  res.print_stats(n, sizeof(T));
  logger.log(kV.csv_name, "RAM", n, o.grade, 0, res, sizeof(T));
  if (!o.out.empty() && !write_raw(o.out, y.data(), n)) {
    std::cerr << "Error: could not write " << o.out << std::endl;
    return 1;
  }
  if (!o.verify) return 0;
  // the serial loop against direct window sums at a few frames
  size_t bad = 0;
  const size_t frames = n / C;
  for (size_t f : {(size_t)0, frames / 3, frames / 2, frames - 1}) {
    if (f >= frames) continue;
    for (int c = 0; c < C; ++c) {
      int64_t s = 0;
      for (long long j = (long long)f - o.grade + 1; j <= (long long)f; ++j)
        if (j >= 0) s += (int64_t)x[(size_t)j * C + c];
      const double e = sizeof(T) == 2 ? (double)(T)(s / o.grade) : (double)(float)((double)s / o.grade);
      bad += (double)y[f * C + c] != e;
    }
  }
  std::cout << "VERIFY: " << bad << " mismatches" << std::endl;
  return bad == 0 ? 0 : 2;
}

int run_synthetic(const Options& o) {
  if (kV.algo < 0)
    return o.dtype == MAVG_F32 ? run_cpu_synthetic<float>(o) : run_cpu_synthetic<int16_t>(o);
  return o.dtype == MAVG_F32 ? run_gpu_synthetic<float>(o) : run_gpu_synthetic<int16_t>(o);
}

bool parse_int(const char* s, int& v) {
  try {
    size_t pos = 0;
    v = std::stoi(s, &pos);
    return pos == std::string(s).size();
  } catch (...) {
    return false;
  }
}

}  // namespace

int main(int argc, char* argv[]) {
  if (argc < 4) {
    std::cerr << "Usage: " << argv[0] << " <wav_path> <grade> <block_size>"
              << " [--out <wav>] [--modes standard|unified|both] [--csv <file>]\n"
              << "       " << argv[0] << " - <grade> <block_size> --synthetic <n_samples>"
              << " [--dtype f32|i16] [--channels C] [--seed S] [--verify] [--csv <file>]" << std::endl;
    return 1;
  }
  Options o;
  o.wav = argv[1];
  if (!parse_int(argv[2], o.grade) || !parse_int(argv[3], o.block)) {
    std::cerr << "Error: grade and block size must be integers" << std::endl;
    return 1;
  }
  if (o.block < 32 || o.block > 1024 || o.block % 32 != 0) {
    std::cerr << "Error: Block size must be multiple of 32" << std::endl;
    return 1;
  }
  if (o.grade < 1) {
    std::cerr << "Error: grade must be >= 1" << std::endl;
    return 1;
  }
  for (int i = 4; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "--out" && i + 1 < argc) {
      o.out = argv[++i];
    } else if (a == "--csv" && i + 1 < argc) {
      o.csv = argv[++i];
    } else if (a == "--modes" && i + 1 < argc) {
      const std::string m = argv[++i];
      o.standard = (m == "standard" || m == "both");
      o.unified = (m == "unified" || m == "both");
      if (!o.standard && !o.unified) {
        std::cerr << "Error: --modes standard|unified|both" << std::endl;
        return 1;
      }
    } else if (a == "--synthetic" && i + 1 < argc) {
      const long long v = std::atoll(argv[++i]);
      if (v < 1) {
        std::cerr << "Error: --synthetic needs a sample count >= 1" << std::endl;
        return 1;
      }
      o.synth_n = (size_t)v;
    } else if (a == "--dtype" && i + 1 < argc) {
      const std::string d = argv[++i];
      if (d != "f32" && d != "i16") {
        std::cerr << "Error: --dtype f32|i16" << std::endl;
        return 1;
      }
      o.dtype = d == "f32" ? MAVG_F32 : MAVG_I16;
    } else if (a == "--channels" && i + 1 < argc) {
      if (!parse_int(argv[++i], o.channels) || o.channels < 1) {
        std::cerr << "Error: --channels needs an integer >= 1" << std::endl;
        return 1;
      }
    } else if (a == "--seed" && i + 1 < argc) {
      o.seed = std::strtoull(argv[++i], nullptr, 0);
    } else if (a == "--verify") {
      o.verify = true;
    } else {
      std::cerr << "Error: unknown option " << a << std::endl;
      return 1;
    }
  }
  if (o.synth_n > 0) {
    if (o.synth_n < (size_t)o.channels) {
      std::cerr << "Error: --synthetic needs at least one frame" << std::endl;
      return 1;
    }
    return run_synthetic(o);
  }
  if (o.verify) {
    std::cerr << "Error: --verify applies to --synthetic runs" << std::endl;
    return 1;
  }
  WavInfo info;
  std::vector<int16_t> samples;
  const std::string err = read_wav_i16(o.wav, info, samples);
  if (!err.empty()) {
    std::cout << err << std::endl;
    return 1;
  }
  if (samples.empty()) {
    std::cout << "no samples" << std::endl;
    return 1;
  }
  std::vector<int16_t> out(samples.size(), 0);
  const int rc = kV.algo < 0 ? run_cpu(o, info.channels, samples, out) : run_gpu(o, info.channels, samples, out);
  if (rc == 0 && !o.out.empty() && !write_wav_i16(o.out, info, out)) {
    std::cerr << "Error: could not write " << o.out << std::endl;
    return 1;
  }
  return rc;
}
