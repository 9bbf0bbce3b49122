// mavg_direct.hip -- direct LDS-tiled and naive kernel instantiations.
#include "mavg_launch.hpp"

namespace mavg {

int direct_any(int dtype, bool wide, int C, int width, const void* in, void* out, const void* hist,
               long long nframes, int k, hipStream_t st) {
  if (dtype == MAVG_F32) return dispatch_direct<float, double>(C, width, in, out, hist, nframes, k, st);
  if (wide) return dispatch_direct<int16_t, int64_t>(C, width, in, out, hist, nframes, k, st);
  return dispatch_direct<int16_t, int32_t>(C, width, in, out, hist, nframes, k, st);
}

int naive_any(int dtype, bool wide, const void* in, void* out, const void* hist, long long nframes, int C, int k,
              hipStream_t st) {
  if (dtype == MAVG_F32) return launch_naive<float, double>(in, out, hist, nframes, C, k, st);
  if (wide) return launch_naive<int16_t, int64_t>(in, out, hist, nframes, C, k, st);
  return launch_naive<int16_t, int32_t>(in, out, hist, nframes, C, k, st);
}

}  // namespace mavg
