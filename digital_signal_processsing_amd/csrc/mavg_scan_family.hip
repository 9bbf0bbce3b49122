// mavg_scan_family.hip -- per-dtype channel switch of the scan family; the
// instantiations themselves come from mavg_scan_inst.hip objects.
#include "mavg_launch.hpp"

namespace mavg {

#define MAVG_EXTERN_C(T, A)                                                                                    \
  extern template int dispatch_scan_c<T, A, 1>(bool, bool, const Sig&, int, int, hipStream_t, Workspace);                                                  \
  extern template int dispatch_scan_c<T, A, 2>(bool, bool, const Sig&, int, int, hipStream_t, Workspace);                                                  \
  extern template int dispatch_scan_c<T, A, 3>(bool, bool, const Sig&, int, int, hipStream_t, Workspace);                                                  \
  extern template int dispatch_scan_c<T, A, 4>(bool, bool, const Sig&, int, int, hipStream_t, Workspace);                                                  \
  extern template int dispatch_scan_c<T, A, 5>(bool, bool, const Sig&, int, int, hipStream_t, Workspace);                                                  \
  extern template int dispatch_scan_c<T, A, 6>(bool, bool, const Sig&, int, int, hipStream_t, Workspace);                                                  \
  extern template int dispatch_scan_c<T, A, 7>(bool, bool, const Sig&, int, int, hipStream_t, Workspace);                                                  \
  extern template int dispatch_scan_c<T, A, 8>(bool, bool, const Sig&, int, int, hipStream_t, Workspace);

MAVG_EXTERN_C(float, double)
MAVG_EXTERN_C(int16_t, int32_t)
MAVG_EXTERN_C(int16_t, int64_t)

int scan_f32(int C, bool vec, bool hs, const Sig& sg, int k, int block, hipStream_t st, Workspace ws) {
  return dispatch_scan<float, double>(C, vec, hs, sg, k, block, st, ws);
}
int scan_i16(int C, bool vec, bool hs, const Sig& sg, int k, int block, hipStream_t st, Workspace ws) {
  return dispatch_scan<int16_t, int32_t>(C, vec, hs, sg, k, block, st, ws);
}
int scan_i16_wide(int C, bool vec, bool hs, const Sig& sg, int k, int block, hipStream_t st, Workspace ws) {
  return dispatch_scan<int16_t, int64_t>(C, vec, hs, sg, k, block, st, ws);
}

}  // namespace mavg
