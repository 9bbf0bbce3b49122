#!/bin/bash
# Tile-shape sweep over window sizes for fp32 mono, int16 mono and int16
# stereo: the data behind dispatch_scan_f's rules (DESIGN.md "Tuning").
# A variant whose LDS need exceeds the budget prints "launch failed" and is
# skipped by the filter of the next run.  Run on the GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/sweep_shapes; mkdir -p $OUT
run() { # tag args...
  local tag=$1; shift
  timeout -k 10 150 tools/tune/tune_scan "$@" > $OUT/$tag.log 2>&1
  local rc=$?
  [ $rc -ge 124 ] && { echo "FATAL $rc in $tag"; exit $rc; }
  return 0
}
for k in 64 512 1024 2048 4096 8192 16384; do
  run f32_k$k 30 $k 8 f32 10 "copy flat|tile U1 NT0 remap64|tile U2 NT|tile U4 NT|tile U8 NT|seg rule|f32 product"
done
for k in 8192 16384; do
  run i16C1_k$k 30 $k 8 i16 10 "copy flat|tile|seg rule|product" 1
  run i16C2_k$k 30 $k 8 i16 10 "copy flat|U2 NT0|U4 NT0|seg rule|product" 2
done
echo sweep done
