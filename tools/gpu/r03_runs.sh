#!/bin/bash
# Run totals in the look-ahead carry (window-matched runs): parity incl. forced
# schedules and the debug build, then A/B: 64-tile runs (abl/libmavg_g64.so),
# window-matched runs without run totals (abl/libmavg_noruns.so), with them (libmavg.so)
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03r}
mkdir -p $OUT
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_parity.py tests/test_debug_build.py -x -q --timeout 200 --timeout-method thread \
  -k "period_remap or ahead_records_bitwise or hillis_long or debug_build or ahead_window_edges or ahead_short" > $OUT/pytest_runs.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_runs.log; [ $rc -eq 0 ] || exit $rc
for cfg in "--k 1000000 --c 1 --dtype f32" "--k 4000000 --c 1 --dtype f32" "--k 2000000 --c 1 --dtype f32" \
           "--k 600000 --c 1 --dtype f32" "--k 1000000 --c 2 --dtype i16" "--k 1500000 --c 1 --dtype i16"; do
  $T 180 python -u tools/tune/ab_libs.py abl/libmavg_g64.so abl/libmavg_noruns.so digital_signal_processsing_amd/lib/libmavg.so abl/libmavg_runs5.so \
     $cfg --rounds 4 --steps 10 >> $OUT/ab.log 2>&1 || { echo "ab failed: $cfg"; exit 1; }
  tail -6 $OUT/ab.log | head -5 | cut -c1-150
done
