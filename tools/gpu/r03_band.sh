#!/bin/bash
# Row-band scan: long-window parity tests, then an in-process A/B against the round-2 look-ahead library (abl/)
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03h}
mkdir -p $OUT
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread \
  -k "ahead or long_window or rounding or unaligned_and_large or long_2p30 or i16_stereo_2p30 or dispatch_boundaries" > $OUT/pytest_long.log 2>&1
echo "pytest rc=$?"; tail -3 $OUT/pytest_long.log
for cfg in "--k 44100 --c 1 --dtype f32" "--k 44100 --c 2 --dtype i16" "--k 20000 --c 1 --dtype f32" \
           "--k 100000 --c 2 --dtype i16" "--k 8200 --c 1 --dtype f32"; do
  $T 180 python -u tools/tune/ab_libs.py abl/libmavg_ahead.so digital_signal_processsing_amd/lib/libmavg.so \
     $cfg --rounds 4 --steps 10 >> $OUT/ab.log 2>&1 || { echo "ab failed: $cfg"; break; }
  tail -4 $OUT/ab.log | cut -c1-150
done
