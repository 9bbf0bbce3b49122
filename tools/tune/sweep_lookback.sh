#!/bin/bash
# Look-back tile scan vs the halo-staged tile scan over window sizes (fp32
# mono, int16 mono, int16 stereo): where dispatch_scan_f switches.  GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/sweep_lookback; mkdir -p $OUT
run() { local tag=$1; shift; timeout -k 10 150 tools/tune/tune_scan "$@" > $OUT/$tag.log 2>&1; local rc=$?; [ $rc -ge 124 ] && { echo "FATAL $rc in $tag"; exit $rc; }; [ $rc -ne 0 ] && echo "rc=$rc in $tag"; return 0; }
for k in 1024 2048 4096 8192 16384 44100 200000; do
  run f32_k$k 30 $k 8 f32 10 "copy flat|lookback|tile U2 NT0|tile U4 NT0|tile U8 NT0|f32 product"
  run i16C1_k$k 30 $k 8 i16 10 "copy flat|lookback|U4 NT3|U4 NT0|U8 NT0|product" 1
  run i16C2_k$k 30 $k 8 i16 10 "copy flat|lookback|U4 NT3|U4 NT0|product" 2
done
echo sweep done
