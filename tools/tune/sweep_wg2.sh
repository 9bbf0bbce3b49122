#!/bin/bash
# 1024-thread tiles with up to 80 KiB of LDS vs the segment scan at windows
# whose halo is 16-64 KiB.  GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/sweep_wg2; mkdir -p $OUT
run() { local tag=$1; shift; timeout -k 10 150 tools/tune/tune_scan "$@" > $OUT/$tag.log 2>&1; local rc=$?; [ $rc -ge 124 ] && { echo "FATAL $rc in $tag"; exit $rc; }; return 0; }
run f32_k8192 30 8192 8 f32 10 "copy flat|tileX U2 nt0 wg1024|tileX U1 nt0 wg1024|tileX U2 nt0 wg512|seg rule|f32 product"
run f32_k12000 30 12000 8 f32 10 "copy flat|tileX U2 nt0 wg1024|tileX U1 nt0 wg1024|seg rule|f32 product"
run i16C1_k16384 30 16384 8 i16 10 "copy flat|wg1024|U2 wg512|seg rule|product" 1
run i16C1_k24000 30 24000 8 i16 10 "copy flat|wg1024|seg rule|product" 1
run i16C2_k8192 30 8192 8 i16 10 "copy flat|wg1024|U2 wg512|seg rule|product" 2
run i16C2_k12000 30 12000 8 i16 10 "copy flat|wg1024|U2 wg512|seg rule|product" 2
echo sweep done
