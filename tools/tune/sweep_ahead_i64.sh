#!/bin/bash
# int16 windows > 65535 frames (int64 carry): look-ahead tile shape per window.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/sweep_ahead_i64; mkdir -p $OUT
for k in ${KSI:-100000 441000}; do
  for C in 1 2; do
    timeout -k 10 150 tools/tune/tune_scan 30 $k 6 i16 10 "copy flat|product|i64" $C > $OUT/i16C${C}_k$k.log 2>&1 || { echo "rc=$? k=$k C=$C"; exit 1; }
    tail -7 $OUT/i16C${C}_k$k.log
  done
done
echo sweep done
