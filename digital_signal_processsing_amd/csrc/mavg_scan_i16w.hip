// mavg_scan_i16w.hip -- streaming-scan instantiations for int16_t samples, int64_t accumulation.
#include "mavg_launch.hpp"

namespace mavg {

int scan_i16_wide(int C, bool vec, bool hs, const void* in, void* out, const void* hist, long long nframes, int k,
           hipStream_t st) {
  return dispatch_scan<int16_t, int64_t>(C, vec, hs, in, out, hist, nframes, k, st);
}

}  // namespace mavg
