#!/bin/bash
# Look-ahead (one HBM pass) vs two-pass look-back vs the 1024-thread tile at long windows.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/sweep_ahead; mkdir -p $OUT
run() { local tag=$1; shift; timeout -k 10 150 tools/tune/tune_scan "$@" > $OUT/$tag.log 2>&1; local rc=$?; [ $rc -ge 124 ] && { echo "FATAL $rc in $tag"; exit $rc; }; [ $rc -ne 0 ] && echo "rc=$rc in $tag"; tail -25 $OUT/$tag.log; return 0; }
for k in ${KS:-44100 16384 200000}; do
  run f32_k$k 30 $k 5 f32 10 "copy flat|lookback U2|ahead|f32 product"
done
for k in ${KSI:-44100}; do
  run i16C1_k$k 30 $k 6 i16 10 "copy flat|i16 lookback U2|i16 ahead|product" 1
  run i16C2_k$k 30 $k 6 i16 10 "copy flat|stereo lookback U2|stereo ahead|product" 2
done
echo sweep done
