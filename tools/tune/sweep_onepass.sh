#!/bin/bash
# One-pass look-back vs the two-pass look-back / 1024-thread tiles at long
# windows, and the split nt-load policy of the tile scan at the headline
# windows.  Every GPU step has its own time limit; a fatal exit ends the sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/sweep_onepass; mkdir -p $OUT
run() { local tag=$1; shift; echo "== $tag"; timeout -k 10 150 tools/tune/tune_scan "$@" > $OUT/$tag.log 2>&1; local rc=$?; tail -n 20 $OUT/$tag.log; [ $rc -ge 124 ] && { echo "FATAL $rc in $tag"; exit $rc; }; [ $rc -ne 0 ] && echo "rc=$rc in $tag"; return 0; }
run f32_k44100 30 44100 6 f32 10 "copy flat|lookback|onepass|f32 product"
run f32_k16384 30 16384 6 f32 10 "copy flat|lookback|onepass|f32 product"
run f32_k200000 30 200000 6 f32 10 "copy flat|lookback|onepass|f32 product"
run f32_k1024_split 30 1024 10 f32 10 "copy flat|tileS"
run f32_k4096_split 30 4096 10 f32 10 "copy flat|tileS"
run i16C2_k44100 30 44100 6 i16 10 "copy flat|stereo lookback|stereo onepass|stereo product" 2
run i16C1_k44100 30 44100 6 i16 10 "copy flat|i16 lookback|i16 onepass|i16 product" 1
run i16C2_k1024_split 30 1024 10 i16 10 "copy flat|stereo tileS" 2
run i16C1_k1024_split 30 1024 10 i16 10 "copy flat|i16 tileS" 1
echo sweep done
