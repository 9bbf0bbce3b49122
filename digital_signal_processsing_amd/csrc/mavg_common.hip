// mavg_common.hip -- per-device attribute cache and output-conversion
// parameters shared by every kernel family.
#include "mavg_launch.hpp"

namespace mavg {

thread_local LaunchPlan* g_plan = nullptr;
#ifdef MAVG_TEST_HOOKS
std::atomic<int> g_test_ahead_slots{-1};
std::atomic<int> g_test_ahead_spin{-1};
#endif

// ---- per-device attribute cache (no stream work, capture-safe) --------------
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
  o.inv_up = o.inv_k * (1.0 + 0x1p-50);  // to_out_i16: the product stays above S/k by < 2^-48 relative
  if (k >= 2 && k <= 65535) {  // to_out_i16_magic
    int l = 0;
    while ((1LL << l) < (long long)k) ++l;  // 2^l >= k > 2^(l-1)
    o.magic = (uint32_t)(((uint64_t)1 << (31 + l)) / (uint64_t)k + 1);
    o.shift = l - 1;
  }
  return o;
}

}  // namespace mavg

#ifdef MAVG_TEST_HOOKS
// include/mavg_debug.h: exported by the debug build (lib/libmavg_debug.so) only
extern "C" int mavg_test_ahead_schedule(int slots, int spin) {
  mavg::g_test_ahead_slots.store(slots < 0 ? -1 : std::min(slots, 1 << 30), std::memory_order_relaxed);
  mavg::g_test_ahead_spin.store(spin < 0 ? -1 : std::min(spin, 1 << 20), std::memory_order_relaxed);
  return MAVG_OK;
}
#endif
