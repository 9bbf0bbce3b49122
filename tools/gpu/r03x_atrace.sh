#!/bin/bash
# phase timeline of the look-ahead scan (MAVG_AHEAD_TRACE build abl/libmavg_atrace.so, tools/tune/ahead_trace.py)
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03x_atrace}
mkdir -p $OUT
for cfg in "--k 44100 --c 1 --dtype f32" "--k 44100 --c 2 --dtype i16" "--k 44100 --c 1 --dtype i16" \
           "--k 44100 --c 1 --dtype f32 --algo 3" "--k 1000000 --c 1 --dtype f32" "--k 4000000 --c 1 --dtype f32"; do
  echo "== $cfg" >> $OUT/trace.log
  timeout -k 10 120 python -u tools/tune/ahead_trace.py abl/libmavg_atrace.so $cfg >> $OUT/trace.log 2>&1 || { echo "trace failed: $cfg"; exit 1; }
done
grep -v amdgpu.ids $OUT/trace.log | cut -c1-150
