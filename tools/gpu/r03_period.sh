#!/bin/bash
# Window-matched XCD runs for windows past the L2 reach: parity, then A/B of
# the fixed 64-tile runs (abl/libmavg_g64.so), window-matched runs at D = 1024 (libmavg.so), 512 and 768 (abl/libmavg_pd*.so)
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03p}
mkdir -p $OUT
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "period_remap or grouped_xcd or ahead_records_bitwise" > $OUT/pytest_period.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_period.log; [ $rc -eq 0 ] || exit $rc
for cfg in "--k 1000000 --c 1 --dtype f32" "--k 4000000 --c 1 --dtype f32" "--k 600000 --c 1 --dtype f32" \
           "--k 1000000 --c 2 --dtype i16" "--k 2000000 --c 1 --dtype f32" "--k 1500000 --c 1 --dtype i16"; do
  $T 180 python -u tools/tune/ab_libs.py abl/libmavg_g64.so digital_signal_processsing_amd/lib/libmavg.so abl/libmavg_pd512.so abl/libmavg_pd768.so \
     $cfg --rounds 4 --steps 10 >> $OUT/ab.log 2>&1 || { echo "ab failed: $cfg"; exit 1; }
  tail -6 $OUT/ab.log | head -5 | cut -c1-150
done
