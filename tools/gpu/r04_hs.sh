#!/bin/bash
# Round 4: the Hillis-Steele look-ahead tile by LDS-DMA (release) against the
# register-staged round-3 form (lib/libmavg_hsnodma.so, -DMAVG_HS_NODMA), in
# bench.py's timing (tools/tune/ab_libs.py), outputs compared bit for bit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r04_hs}
mkdir -p "$OUT"
L=digital_signal_processsing_amd/lib
for spec in "44100 1 f32 2" "20000 1 f32 2" "44100 2 i16 0"; do
  read -r k c dt dist <<< "$spec"
  timeout -k 10 200 python -u tools/tune/ab_libs.py $L/libmavg_hsnodma.so $L/libmavg.so --k "$k" --c "$c" \
    --dtype "$dt" --dist "$dist" --algo 3 --rounds 6 > "$OUT/hs_${dt}_c${c}_k${k}.log" 2>&1
  rc=$?
  cat "$OUT/hs_${dt}_c${c}_k${k}.log"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
