// wav_io.hpp -- 16-bit PCM WAV reader/writer for the bin_* CLIs.
//
// Counterpart of the reference's wav_header.h (extractSamples :26-48,
// writeSamples :50-60).  Accepts every file the reference accepts (the
// canonical 44-byte header scipy.io.wavfile writes) and additionally walks
// RIFF chunks (LIST/fact chunks before "data"), reads the payload in one
// bulk read instead of one sample at a time, and rejects anything that is not
// 16-bit integer PCM (the reference rejects 8/24/32/64-bit, :31-34).
#pragma once

#include <cstdint>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

namespace mavg_cli {

struct WavInfo {
  uint16_t channels = 0;
  uint32_t sample_rate = 0;
  uint16_t bits = 0;
  uint32_t data_bytes = 0;
};

inline uint32_t rd32(const unsigned char* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }
inline uint16_t rd16(const unsigned char* p) { return (uint16_t)(p[0] | (p[1] << 8)); }

// Returns an empty string on success, else the reason.
inline std::string read_wav_i16(const std::string& path, WavInfo& info, std::vector<int16_t>& samples) {
  std::ifstream in(path, std::ios::binary);
  if (!in) return "could not open file";
  unsigned char riff[12];
  if (!in.read(reinterpret_cast<char*>(riff), 12)) return "file too short for a RIFF header";
  if (std::memcmp(riff, "RIFF", 4) != 0 || std::memcmp(riff + 8, "WAVE", 4) != 0) return "not a RIFF/WAVE file";
  bool have_fmt = false;
  uint16_t format = 0;
  for (;;) {
    unsigned char ch[8];
    if (!in.read(reinterpret_cast<char*>(ch), 8)) return "no data chunk";
    const uint32_t size = rd32(ch + 4);
    if (std::memcmp(ch, "fmt ", 4) == 0) {
      if (size < 16) return "fmt chunk too short";
      if (size > (1u << 20)) return "fmt chunk too large";
      std::vector<unsigned char> f(size);
      if (!in.read(reinterpret_cast<char*>(f.data()), size)) return "truncated fmt chunk";
      format = rd16(f.data());
      info.channels = rd16(f.data() + 2);
      info.sample_rate = rd32(f.data() + 4);
      info.bits = rd16(f.data() + 14);
      have_fmt = true;
      if (size & 1) in.ignore(1);
    } else if (std::memcmp(ch, "data", 4) == 0) {
      if (!have_fmt) return "data chunk before fmt chunk";
      if (info.bits != 16) return "unsupported bits per sample: " + std::to_string(info.bits);
      if (format != 1 && format != 0xFFFE) return "not integer PCM (format " + std::to_string(format) + ")";
      if (info.channels == 0) return "zero channels";
      info.data_bytes = size;
      // never allocate more than the file holds (a corrupt size field)
      const std::streampos here = in.tellg();
      in.seekg(0, std::ios::end);
      const std::streamoff remaining = in.tellg() - here;
      in.seekg(here);
      if (remaining < (std::streamoff)size) return "truncated data chunk";
      samples.resize(size / 2);
      if (!in.read(reinterpret_cast<char*>(samples.data()), (std::streamsize)(samples.size() * 2)))
        return "truncated data chunk";
      return "";
    } else {
      in.ignore(size + (size & 1));
    }
  }
}

inline bool write_wav_i16(const std::string& path, const WavInfo& info, const std::vector<int16_t>& samples) {
  std::ofstream out(path, std::ios::binary);
  if (!out) return false;
  const uint32_t data = (uint32_t)(samples.size() * 2);
  unsigned char h[44];
  auto w32 = [&](int o, uint32_t v) { h[o] = v & 255; h[o + 1] = (v >> 8) & 255; h[o + 2] = (v >> 16) & 255; h[o + 3] = v >> 24; };
  auto w16 = [&](int o, uint16_t v) { h[o] = v & 255; h[o + 1] = v >> 8; };
  std::memcpy(h, "RIFF", 4);
  w32(4, 36 + data);
  std::memcpy(h + 8, "WAVEfmt ", 8);
  w32(16, 16);
  w16(20, 1);
  w16(22, info.channels);
  w32(24, info.sample_rate);
  w32(28, info.sample_rate * info.channels * 2);
  w16(32, (uint16_t)(info.channels * 2));
  w16(34, 16);
  std::memcpy(h + 36, "data", 4);
  w32(40, data);
  out.write(reinterpret_cast<const char*>(h), 44);
  out.write(reinterpret_cast<const char*>(samples.data()), data);
  return (bool)out;
}

}  // namespace mavg_cli
