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
#include <algorithm>
#include <cstdint>
#include <cstdlib>
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
};

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
  if (kV.banner) {
    std::cout << kV.banner << std::endl;
    std::cout << "Samples: " << samples.size() << std::endl;
    std::cout << "point: " << o.grade << std::endl;
    std::cout << "block Size: " << o.block << std::endl;
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
              << " [--out <wav>] [--modes standard|unified|both] [--csv <file>]" << std::endl;
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
    } else {
      std::cerr << "Error: unknown option " << a << std::endl;
      return 1;
    }
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
