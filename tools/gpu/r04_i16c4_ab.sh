#!/bin/bash
# Round 4: int16 4 channels past the wide tile, the wide look-ahead (release)
# against the unit look-ahead (lib/libmavg_noi16w.so, -DMAVG_NO_I16C4_WIDE_AHEAD),
# in bench.py's timing (tools/tune/ab_libs.py), outputs compared bit for bit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r04_i16c4_ab}
mkdir -p "$OUT"
L=digital_signal_processsing_amd/lib
for k in 44100 20000 60000; do
  timeout -k 10 200 python -u tools/tune/ab_libs.py $L/libmavg_noi16w.so $L/libmavg.so --k "$k" --c 4 \
    --dtype i16 --rounds 8 > "$OUT/bench_timing_i16_c4_k${k}.log" 2>&1
  rc=$?
  cat "$OUT/bench_timing_i16_c4_k${k}.log"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
