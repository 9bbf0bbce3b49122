#!/bin/bash
# Round 4: fp32 8 channels, the halo-only chan tile (XG, release) against the
# staged chan tile (lib/libmavg_noxg.so, -DMAVG_NO_CHAN_XG) in bench.py's
# timing; then the in-process tuner for 4 channels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r04_xg_ab}
mkdir -p "$OUT"
L=digital_signal_processsing_amd/lib
for k in 1024 768 512; do
  timeout -k 10 200 python -u tools/tune/ab_libs.py $L/libmavg_noxg.so $L/libmavg.so --k "$k" --c 8 \
    --dtype f32 --dist 2 --rounds 8 > "$OUT/bench_timing_xg_c8_k${k}.log" 2>&1
  rc=$?
  cat "$OUT/bench_timing_xg_c8_k${k}.log"
  [ $rc -ne 0 ] && exit $rc
done
for k in 1024 2048; do
  timeout -k 10 150 tools/tune/wide_ab 30 $k 4 6 1 f32 > "$OUT/xg_c4_k$k.log" 2>&1 || exit $?
  cat "$OUT/xg_c4_k$k.log"
done
exit 0
