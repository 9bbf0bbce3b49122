#!/bin/bash
# One-pass vs two-pass look-back vs the segment / tile scans at long windows.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/sweep_lookback2; mkdir -p $OUT
run() { local tag=$1; shift; timeout -k 10 150 tools/tune/tune_scan "$@" > $OUT/$tag.log 2>&1; local rc=$?; [ $rc -ge 124 ] && { echo "FATAL $rc in $tag"; exit $rc; }; [ $rc -ne 0 ] && echo "rc=$rc in $tag"; return 0; }
for k in 4096 8192 16384 44100 200000; do
  run f32_k$k 30 $k 8 f32 10 "copy flat|lookback|seg rule|tile U8 NT0|f32 product"
  run i16C1_k$k 30 $k 8 i16 10 "copy flat|lookback|seg rule|U8 NT0|product" 1
  run i16C2_k$k 30 $k 8 i16 10 "copy flat|lookback|seg rule|U4 NT0|product" 2
done
echo sweep done
