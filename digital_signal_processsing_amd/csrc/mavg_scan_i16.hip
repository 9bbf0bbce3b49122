// mavg_scan_i16.hip -- streaming-scan instantiations for int16_t samples, int32_t accumulation.
#include "mavg_launch.hpp"

namespace mavg {

int scan_i16(int C, bool vec, bool hs, const void* in, void* out, const void* hist, long long nframes, int k,
           hipStream_t st) {
  return dispatch_scan<int16_t, int32_t>(C, vec, hs, in, out, hist, nframes, k, st);
}

}  // namespace mavg
