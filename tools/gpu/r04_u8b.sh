#!/bin/bash
# Round 4: fp32 mono 8192-frame tiles, both harnesses on one box: bench.py's
# timing (ab_libs.py, release vs -DMAVG_AHEAD_NO_U8) and the in-process tuner.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r04_u8b}
mkdir -p "$OUT"
L=digital_signal_processsing_amd/lib
for spec in "44100 1 f32 2" "2000000 1 f32 2" "44100 1 f32 1"; do
  read -r k c dt dist <<< "$spec"
  timeout -k 10 200 python -u tools/tune/ab_libs.py $L/libmavg_u4.so $L/libmavg.so --k "$k" --c "$c" \
    --dtype "$dt" --dist "$dist" --rounds 12 > "$OUT/u8_${dt}_c${c}_k${k}_d${dist}.log" 2>&1
  rc=$?
  cat "$OUT/u8_${dt}_c${c}_k${k}_d${dist}.log"
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 150 tools/tune/wide_ab 30 44100 1 6 1 f32 > "$OUT/wide_ab_k44100.log" 2>&1 || exit $?
cat "$OUT/wide_ab_k44100.log"
exit 0
