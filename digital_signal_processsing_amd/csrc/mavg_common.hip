// mavg_common.hip -- per-device attribute cache and output-conversion
// parameters shared by every kernel family.
#include "mavg_launch.hpp"

namespace mavg {

thread_local LaunchPlan* g_plan = nullptr;
std::atomic<int> g_test_ahead_slots{-1};
std::atomic<int> g_test_ahead_spin{-1};

// ---- per-device attribute cache (no stream work, capture-safe) --------------
constexpr int kMaxDevices = 64;
static std::atomic<int> g_cu_count[kMaxDevices];

int device_cu_count() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return 256;
  int v = g_cu_count[dev].load(std::memory_order_relaxed);
  if (v > 0) return v;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  g_cu_count[dev].store(cus, std::memory_order_relaxed);
  return cus;
}

OutParams make_out_params(int k) {
  OutParams o{};
  o.k = k;
  o.inv_k = 1.0 / (double)k;
  if (k >= 2) {
    int l = 0;
    while ((1LL << l) < (long long)k) ++l;                  // l = ceil(log2 k), 2^l >= k > 2^(l-1)
    const uint64_t m = ((uint64_t)1 << (31 + l)) / (uint64_t)k + 1;  // < 2^32 for k <= 65535
    o.magic = (uint32_t)m;
    o.shift = l - 1;
  } else {
    o.magic = 0;
    o.shift = 0;
  }
  return o;
}

}  // namespace mavg

extern "C" int mavg_test_ahead_schedule(int slots, int spin) {
  mavg::g_test_ahead_slots.store(slots < 0 ? -1 : std::min(slots, 1 << 30), std::memory_order_relaxed);
  mavg::g_test_ahead_spin.store(spin < 0 ? -1 : std::min(spin, 1 << 20), std::memory_order_relaxed);
  return MAVG_OK;
}
