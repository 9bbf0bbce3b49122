#!/bin/bash
# Per-tile records (product, pf=4) vs per-wave records (the earlier form,
# tools/tune/ahead_wave_records.hpp), in one process per window.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/sweep_records; mkdir -p $OUT
run() { local tag=$1; shift; timeout -k 10 150 tools/tune/tune_scan "$@" > $OUT/$tag.log 2>&1 || { echo "rc=$? $tag"; exit 1; }; echo "== $tag"; grep -E "copy flat|product|rc pf|records" $OUT/$tag.log | grep -v recomputes; }
for k in 8192 44100; do run f32_k$k 30 $k 6 f32 10 "copy flat|product|rc pf"; done
for k in 30000 44100; do
  run i16C1_k$k 30 $k 6 i16 10 "copy flat|product|rc pf|tile-records" 1
  run i16C2_k$k 30 $k 6 i16 10 "copy flat|product|rc pf|tile-records" 2
done
echo sweep done
