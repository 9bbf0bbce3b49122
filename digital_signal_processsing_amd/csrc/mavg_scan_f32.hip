// mavg_scan_f32.hip -- streaming-scan instantiations for float samples, double accumulation.
#include "mavg_launch.hpp"

namespace mavg {

int scan_f32(int C, bool vec, bool hs, const void* in, void* out, const void* hist, long long nframes, int k,
           hipStream_t st) {
  return dispatch_scan<float, double>(C, vec, hs, in, out, hist, nframes, k, st);
}

}  // namespace mavg
