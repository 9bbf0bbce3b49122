#!/bin/bash
# Hillis-Steele flavour: tile shape x cache policy across windows (and a few
# Blelloch shapes under the split policy).  Each GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/sweep_hillis; mkdir -p $OUT
run() { local tag=$1; shift; echo "== $tag"; timeout -k 10 150 tools/tune/tune_scan "$@" > $OUT/$tag.log 2>&1; local rc=$?; tail -n 20 $OUT/$tag.log; [ $rc -ge 124 ] && { echo "FATAL $rc in $tag"; exit $rc; }; [ $rc -ne 0 ] && echo "rc=$rc in $tag"; return 0; }
run f32_k1024 30 1024 8 f32 10 "copy flat|hillisS|tileS U2 nt13 wg256|tileS U4 nt13 wg256|tileS U2 nt3 wg256|tileS U4 nt3 wg256"
run f32_k64 30 64 8 f32 10 "copy flat|hillisS|tileS U2 nt13 wg256|tileS U2 nt3 wg256|tileS U4 nt3 wg256|tileS U4 nt13 wg256"
run f32_k4096 30 4096 8 f32 10 "copy flat|hillisS|f32 product"
run i16C1_k1024 30 1024 8 i16 10 "copy flat|i16 hillisS|i16 product" 1
run i16C1_k4096 30 4096 8 i16 10 "copy flat|i16 hillisS|i16 product" 1
run i16C2_k1024 30 1024 8 i16 10 "copy flat|stereo hillisS|stereo product" 2
run i16C2_k4096 30 4096 8 i16 10 "copy flat|stereo hillisS|stereo product" 2
echo sweep done
