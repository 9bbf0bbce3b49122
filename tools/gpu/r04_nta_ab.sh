#!/bin/bash
# Round 4: phase A non-temporal for fp32 8192-frame look-ahead tiles (release)
# against the default policy (lib/libmavg_nonta.so, -DMAVG_AHEAD_NO_NTA), in
# bench.py's timing (tools/tune/ab_libs.py), outputs compared bit for bit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r04_nta_ab}
mkdir -p "$OUT"
L=digital_signal_processsing_amd/lib
for k in 4000000 2000000 1000000 600000; do
  timeout -k 10 200 python -u tools/tune/ab_libs.py $L/libmavg_nonta.so $L/libmavg.so --k "$k" --c 1 \
    --dtype f32 --dist 2 --rounds 8 > "$OUT/nta_f32_k${k}.log" 2>&1
  rc=$?
  cat "$OUT/nta_f32_k${k}.log"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
