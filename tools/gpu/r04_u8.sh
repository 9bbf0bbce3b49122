#!/bin/bash
# Round 4: the look-ahead scan's 8192-frame tiles (release) against the round-3
# 4096-frame tiles (lib/libmavg_u4.so, -DMAVG_AHEAD_NO_U8), in bench.py's timing
# (tools/tune/ab_libs.py), outputs compared bit for bit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r04_u8}
mkdir -p "$OUT"
L=digital_signal_processsing_amd/lib
for spec in "44100 1 f32 2" "20000 1 f32 2" "1000000 1 f32 2" "4000000 1 f32 2" "44100 2 i16 0" "100000 2 i16 0"; do
  read -r k c dt dist <<< "$spec"
  timeout -k 10 200 python -u tools/tune/ab_libs.py $L/libmavg_u4.so $L/libmavg.so --k "$k" --c "$c" \
    --dtype "$dt" --dist "$dist" --rounds 8 > "$OUT/u8_${dt}_c${c}_k${k}.log" 2>&1
  rc=$?
  cat "$OUT/u8_${dt}_c${c}_k${k}.log"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
