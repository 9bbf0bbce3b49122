#!/bin/bash
# Look-ahead distance D (MAVG_AHEAD_SLOTS) for the product dispatch, per-tile records.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/sweep_slots; mkdir -p $OUT
for D in 256 512 1024 2048; do
  for w in "f32 8192 1" "f32 44100 1" "i16 44100 1" "i16 44100 2"; do
    set -- $w
    MAVG_AHEAD_SLOTS=$D timeout -k 10 120 tools/tune/tune_scan 30 $2 5 $1 10 "copy flat|product" $3 > $OUT/D${D}_$1_k$2_C$3.log 2>&1 || { echo "rc=$? D=$D $w"; exit 1; }
    printf "D=%-5s %-4s k=%-6s C=%s  " $D $1 $2 $3; grep -E "product" $OUT/D${D}_$1_k$2_C$3.log
  done
done
echo sweep done
