#!/bin/bash
# phase timelines, look-ahead records (abl/libmavg_atrace.so) vs self-published records (libmavg_atrace_self.so)
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03x_atrace2}
mkdir -p $OUT
for lib in abl/libmavg_atrace.so abl/libmavg_atrace_self.so; do
  for cfg in "--k 8192 --c 1 --dtype f32" "--k 44100 --c 1 --dtype f32"; do
    echo "== $lib $cfg" >> $OUT/trace.log
    timeout -k 10 120 python -u tools/tune/ahead_trace.py $lib $cfg >> $OUT/trace.log 2>&1 || { echo "trace failed: $cfg"; exit 1; }
  done
done
grep -v amdgpu.ids $OUT/trace.log | grep -v "^  run [37]" | cut -c1-150
