// mavg_scan_inst.hip -- explicit instantiation of the scan family for one
// (sample type, accumulator, channel count); compiled once per combination
// by the Makefile (-DMAVG_T=... -DMAVG_A=... -DMAVG_C=...) so the build
// parallelises.  The per-dtype switch lives in mavg_scan_family.hip.
#include "mavg_launch.hpp"

namespace mavg {
template int dispatch_scan_c<MAVG_T, MAVG_A, MAVG_C>(bool, bool, const Sig&, int, int, hipStream_t, Workspace);
}  // namespace mavg
