#!/bin/bash
# Prefetched record rounds (pf1 vs pf4) for windows spanning > 256 records.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/sweep_pf; mkdir -p $OUT
for k in 200000 300000 1000000 4000000; do
  timeout -k 10 150 tools/tune/tune_scan 30 $k 5 f32 10 "copy flat|pf|product" > $OUT/f32_k$k.log 2>&1 || { echo "rc=$? f32 k=$k"; exit 1; }
  tail -5 $OUT/f32_k$k.log
done
for k in 600000 2000000; do
  timeout -k 10 150 tools/tune/tune_scan 30 $k 5 i16 10 "copy flat|pf|product" 1 > $OUT/i16_k$k.log 2>&1 || { echo "rc=$? i16 k=$k"; exit 1; }
  tail -5 $OUT/i16_k$k.log
done
echo sweep done
