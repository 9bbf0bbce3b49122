#!/bin/bash
# Group records in the look-ahead scan (very long windows): parity, then A/B against the round-2 library (abl/)
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03j}
mkdir -p $OUT
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "ahead or rounding or unaligned_and_large or int64_division" > $OUT/pytest_long.log 2>&1
echo "pytest rc=$?"; tail -2 $OUT/pytest_long.log
for cfg in "--k 100000 --c 1 --dtype f32" "--k 300000 --c 1 --dtype f32" "--k 1000000 --c 1 --dtype f32" \
           "--k 4000000 --c 1 --dtype f32" "--k 1000000 --c 2 --dtype i16" "--k 44100 --c 1 --dtype f32"; do
  $T 180 python -u tools/tune/ab_libs.py abl/libmavg_ahead.so digital_signal_processsing_amd/lib/libmavg.so \
     $cfg --rounds 4 --steps 10 >> $OUT/ab.log 2>&1 || { echo "ab failed: $cfg"; break; }
  tail -4 $OUT/ab.log | cut -c1-150
done
