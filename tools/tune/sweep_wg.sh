#!/bin/bash
# Workgroup size x tile size at mid-length windows (where halo + tile LDS
# limits occupancy), fp32 mono / int16 mono / int16 stereo.  GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/sweep_wg; mkdir -p $OUT
run() { local tag=$1; shift; timeout -k 10 150 tools/tune/tune_scan "$@" > $OUT/$tag.log 2>&1; local rc=$?; [ $rc -ge 124 ] && { echo "FATAL $rc in $tag"; exit $rc; }; return 0; }
for k in 1024 2048 4096 8192; do
  run f32_k$k 30 $k 8 f32 10 "copy flat|wg|seg rule|f32 product"
  run i16C1_k$k 30 $k 8 i16 10 "copy flat|wg|seg rule|product" 1
  run i16C2_k$k 30 $k 8 i16 10 "copy flat|wg|seg rule|product" 2
done
echo sweep done
