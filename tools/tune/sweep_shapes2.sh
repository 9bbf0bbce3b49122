#!/bin/bash
# Follow-up of sweep_shapes.sh: large windows (tile vs segment boundary).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/sweep_shapes; mkdir -p $OUT
run() { local tag=$1; shift; timeout -k 10 150 tools/tune/tune_scan "$@" > $OUT/$tag.log 2>&1; local rc=$?; [ $rc -ge 124 ] && { echo "FATAL $rc in $tag"; exit $rc; }; return 0; }
for k in 8192 16384; do
  run f32_k$k 30 $k 8 f32 10 "copy flat|tile U4 NT0|tile U8 NT0|seg rule|f32 product"
  run i16C1_k$k 30 $k 8 i16 10 "copy flat|U4 NT0|U8 NT0|seg rule|product" 1
done
for k in 2048 4096 16384; do
  run i16C2_k$k 30 $k 8 i16 10 "copy flat|U2 NT0|U4 NT0|U4 NT3|seg rule|product" 2
done
echo sweep done
