#!/bin/bash
# Hillis-Steele long windows through the look-ahead record carry: parity, then A/B against the round-2 library
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03m}
mkdir -p $OUT
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "hillis or unaligned_and_large or history_equals or golden or ragged or channel_counts" > $OUT/pytest_hs.log 2>&1
echo "pytest rc=$?"; tail -2 $OUT/pytest_hs.log
for cfg in "--k 44100 --c 1 --dtype f32" "--k 44100 --c 2 --dtype i16" "--k 20000 --c 1 --dtype f32"; do
  $T 180 python -u tools/tune/ab_libs.py abl/libmavg_ahead.so digital_signal_processsing_amd/lib/libmavg.so \
     $cfg --algo 3 --rounds 4 --steps 10 >> $OUT/ab.log 2>&1 || { echo "ab failed: $cfg"; break; }
  tail -4 $OUT/ab.log | head -3 | cut -c1-200
done
bash tools/gpu/r03_direct_ab.sh ${1:-r03m}
