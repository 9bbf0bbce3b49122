#!/bin/bash
# Round 4: fp32 8 channels, the channel-per-lane kernels (release) against the
# chunk-per-lane wide kernels (lib/libmavg_nochan.so, -DMAVG_NO_CHAN), in
# bench.py's timing (tools/tune/ab_libs.py), outputs compared.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r04_chan_ab}
mkdir -p "$OUT"
L=digital_signal_processsing_amd/lib
for k in 1024 256 7 4096 44100; do
  timeout -k 10 200 python -u tools/tune/ab_libs.py $L/libmavg_nochan.so $L/libmavg.so --k "$k" --c 8 \
    --dtype f32 --dist 2 --rounds 8 > "$OUT/chan_f32_c8_k${k}.log" 2>&1
  rc=$?
  cat "$OUT/chan_f32_c8_k${k}.log"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
