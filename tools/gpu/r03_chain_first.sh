#!/bin/bash
# Round 3, first GPU pass over the chained look-back scan: its parity tests,
# then an in-process A/B against the round-2 look-ahead library (abl/).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r03a
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "ahead or long_window or rounding or unaligned_and_large or device_synth" \
  > gpurun_out/r03a/pytest_long.log 2>&1
echo "pytest rc=$?" ; tail -5 gpurun_out/r03a/pytest_long.log
for cfg in "--k 44100 --c 1 --dtype f32" "--k 44100 --c 1 --dtype i16" "--k 44100 --c 2 --dtype i16" \
           "--k 1000000 --c 1 --dtype f32" "--k 4000000 --c 1 --dtype f32" "--k 20000 --c 1 --dtype f32" \
           "--k 100000 --c 2 --dtype i16"; do
  $T 180 python -u tools/tune/ab_libs.py abl/libmavg_ahead.so digital_signal_processsing_amd/lib/libmavg.so \
     $cfg --rounds 4 --steps 10 >> gpurun_out/r03a/ab.log 2>&1 || { echo "ab failed: $cfg"; break; }
  tail -4 gpurun_out/r03a/ab.log
done
