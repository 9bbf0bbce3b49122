#!/bin/bash
# self-published records: carry loads after the scan (abl/libmavg_self.so) or before it (libmavg_selfe.so,
# -DMAVG_AHEAD_SELF_EARLY=1) against the release build, fp32 mono windows from 5000 to 44100
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03x_self2}
mkdir -p $OUT
for cfg in "--k 5000 --c 1 --dtype f32" "--k 8192 --c 1 --dtype f32" "--k 12288 --c 1 --dtype f32" "--k 20000 --c 1 --dtype f32" \
           "--k 44100 --c 1 --dtype f32" "--k 20000 --c 2 --dtype i16" "--k 30000 --c 1 --dtype i16"; do
  timeout -k 10 180 python -u tools/tune/ab_libs.py abl/libmavg_cur.so abl/libmavg_self.so abl/libmavg_selfe.so \
     $cfg --rounds 6 --steps 10 >> $OUT/ab.log 2>&1 || { echo "ab failed: $cfg"; exit 1; }
  tail -5 $OUT/ab.log | head -4 | cut -c1-120
done
