// mavg_direct.hip -- direct LDS-tiled and naive kernel instantiations.
#include "mavg_launch.hpp"

namespace mavg {

int direct_any(int dtype, bool wide, int C, int width, const Sig& sg, int k, int block, hipStream_t st) {
  if (dtype == MAVG_F32) return dispatch_direct<float, double>(C, width, sg, k, block, st);
  if (wide) return dispatch_direct<int16_t, int64_t>(C, width, sg, k, block, st);
  return dispatch_direct<int16_t, int32_t>(C, width, sg, k, block, st);
}

int naive_any(int dtype, bool wide, const Sig& sg, int C, int k, int block, hipStream_t st) {
  if (dtype == MAVG_F32) return launch_naive<float, double>(sg, C, k, block, st);
  if (wide) return launch_naive<int16_t, int64_t>(sg, C, k, block, st);
  return launch_naive<int16_t, int32_t>(sg, C, k, block, st);
}

}  // namespace mavg
