#!/bin/bash
# chain-scan phase trace (abl/libmavg_trace.so) + A/B against the round-2 look-ahead library
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03e}
mkdir -p $OUT
T="timeout -k 10"
$T 120 python -u tools/tune/chain_trace.py abl/libmavg_trace.so --k 44100 > $OUT/trace_f32.log 2>&1 && cat $OUT/trace_f32.log
$T 120 python -u tools/tune/chain_trace.py abl/libmavg_trace.so --k 44100 --c 2 --dtype i16 > $OUT/trace_i16s.log 2>&1 && cat $OUT/trace_i16s.log
for cfg in "--k 44100 --c 1 --dtype f32" "--k 44100 --c 2 --dtype i16" "--k 1000000 --c 1 --dtype f32"; do
  $T 180 python -u tools/tune/ab_libs.py abl/libmavg_ahead.so digital_signal_processsing_amd/lib/libmavg.so \
     $cfg --rounds 4 --steps 10 >> $OUT/ab.log 2>&1 || { echo "ab failed: $cfg"; break; }
  tail -4 $OUT/ab.log | cut -c1-150
done
