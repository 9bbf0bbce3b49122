#!/bin/bash
# Round 4: look-ahead phase traces (MAVG_AHEAD_TRACE build, lib/libmavg_atrace.so)
# of the one-second PCM window (int16 stereo, 8192-frame tiles), int16 mono and
# fp32 mono at k=44100, and fp32 k=4e6; then the int16 stereo A/B of record forms.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r04_trace}
mkdir -p "$OUT"
L=digital_signal_processsing_amd/lib/libmavg_atrace.so
for spec in "44100 2 i16" "44100 1 i16" "44100 1 f32" "4000000 1 f32"; do
  read -r k c dt <<< "$spec"
  timeout -k 10 150 python -u tools/tune/ahead_trace.py $L --k "$k" --c "$c" --dtype "$dt" > "$OUT/trace_${dt}_c${c}_k${k}.log" 2>&1
  rc=$?
  cat "$OUT/trace_${dt}_c${c}_k${k}.log"
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 150 tools/tune/wide_ab 30 44100 2 6 1 i16 > "$OUT/records_i16_c2_k44100.log" 2>&1 || exit $?
cat "$OUT/records_i16_c2_k44100.log"
for k in 44100 20000; do  # int16 4 channels past the wide tile: the wide look-ahead against the unit look-ahead
  timeout -k 10 150 tools/tune/wide_ab 30 $k 4 6 1 i16 > "$OUT/wide_i16_c4_k$k.log" 2>&1 || exit $?
  cat "$OUT/wide_i16_c4_k$k.log"
done
exit 0
