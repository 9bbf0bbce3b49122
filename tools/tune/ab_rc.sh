#!/bin/bash
# Focused RC / no-RC A/B on the bench configurations (20 rounds, twice).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/ab_rc; mkdir -p $OUT
run() { local tag=$1; shift; timeout -k 10 200 tools/tune/tune_scan "$@" > $OUT/$tag.log 2>&1; local rc=$?; [ $rc -ge 124 ] && { echo "FATAL $rc in $tag"; exit $rc; }; return 0; }
for rep in 1 2; do
  run f32_k1024_$rep 30 1024 20 f32 10 "copy flat|tile U2 NT0"
  run f32_k4096_$rep 30 4096 20 f32 10 "copy flat|tile U8 NT0"
  run f32_k64_$rep 26 64 20 f32 10 "copy flat|tile U4 NT3|tile U2 NT3"
  run i16C1_k1024_$rep 30 1024 20 i16 10 "copy flat|tile U4 NT3|tile U8 NT0" 1
  run i16C2_k1024_$rep 30 1024 20 i16 10 "copy flat|tile U4 NT3|tile U4 NT0" 2
done
echo ab done
