#!/bin/bash
# After the register diet (carry from a wave scan of the segment totals; RC =
# in-lane prefix rebuilt from LDS after the barrier): tile shapes again, RC
# vs no-RC, fp32 mono / int16 mono / int16 stereo.  GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/sweep_regs; mkdir -p $OUT
run() { local tag=$1; shift; timeout -k 10 150 tools/tune/tune_scan "$@" > $OUT/$tag.log 2>&1; local rc=$?; [ $rc -ge 124 ] && { echo "FATAL $rc in $tag"; exit $rc; }; [ $rc -ne 0 ] && echo "rc=$rc in $tag"; return 0; }
for k in 64 1024 2048 4096; do
  run f32_k$k 30 $k 8 f32 10 "copy flat|tile U|product"
  run i16C1_k$k 30 $k 8 i16 10 "copy flat|i16 tile U|product" 1
  run i16C2_k$k 30 $k 8 i16 10 "copy flat|stereo tile|product" 2
done
echo sweep done
