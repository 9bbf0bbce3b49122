#!/bin/bash
# Load/store cache-policy (NT bits) per tile shape across the windows of the
# dispatch table.  nt: 1 nt stores, 3 nt loads+stores, 4 nt tile loads except
# the tail the next halo re-reads, 5 = 4|1, 13 = 5 + nt halo loads.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/sweep_nt; mkdir -p $OUT
run() { local tag=$1; shift; echo "== $tag"; timeout -k 10 150 tools/tune/tune_scan "$@" > $OUT/$tag.log 2>&1; local rc=$?; tail -n 16 $OUT/$tag.log; [ $rc -ge 124 ] && { echo "FATAL $rc in $tag"; exit $rc; }; [ $rc -ne 0 ] && echo "rc=$rc in $tag"; return 0; }
run f32_k1024 30 1024 8 f32 10 "copy flat|tileS U2 nt0 wg256|tileS U2 nt1 wg256|tileS U2 nt5 wg256|tileS U2 nt13 wg256|f32 product"
run f32_k2048 30 2048 8 f32 10 "copy flat|tileS U2 nt0 wg512|tileS U2 nt1 wg512|tileS U2 nt5 wg512|tileS U2 nt13 wg512|f32 product"
run f32_k4096 30 4096 8 f32 10 "copy flat|tileS U4 nt0 wg512|tileS U4 nt1 wg512|tileS U4 nt5 wg512|tileS U4 nt13 wg512|f32 product"
run f32_k8192 30 8192 8 f32 10 "copy flat|tileS U2 nt0 wg1024|tileS U2 nt1 wg1024|tileS U2 nt5 wg1024|tileS U2 nt13 wg1024|f32 product"
run f32_k44100 30 44100 6 f32 10 "copy flat|lookbackN|f32 product"
run i16C1_k4096 30 4096 8 i16 10 "copy flat|i16 tileS U4 nt0 wg256|i16 tileS U4 nt3 wg256|i16 tileS U4 nt5 wg256|i16 tileS U4 nt13 wg256|i16 product" 1
run i16C1_k8192 30 8192 8 i16 10 "copy flat|i16 tileS U4 nt0 wg512|i16 tileS U4 nt5 wg512|i16 tileS U4 nt13 wg512|i16 product" 1
run i16C1_k16384 30 16384 8 i16 10 "copy flat|i16 tileS U2 nt0 wg1024|i16 tileS U2 nt5 wg1024|i16 tileS U2 nt13 wg1024|i16 product" 1
run i16C2_k2048 30 2048 8 i16 10 "copy flat|stereo tileS U4 nt0 wg256|stereo tileS U4 nt3 wg256|stereo tileS U4 nt5 wg256|stereo tileS U4 nt13 wg256|stereo product" 2
run i16C2_k4096 30 4096 8 i16 10 "copy flat|stereo tileS U4 nt0 wg512|stereo tileS U4 nt5 wg512|stereo tileS U4 nt13 wg512|stereo product" 2
run i16C2_k8192 30 8192 8 i16 10 "copy flat|stereo tileS U2 nt0 wg1024|stereo tileS U2 nt5 wg1024|stereo tileS U2 nt13 wg1024|stereo product" 2
echo sweep done
