#!/bin/bash
# phase A's loads issued after the tile's own and summed after the in-tile scan, the carry's records read
# after the scan (abl/libmavg_latea.so, -DMAVG_AHEAD_LATE_A=1) against the release build, in-process A/B.
# The variant was measured slower and not kept (look-ahead scan).
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03x_latea}
mkdir -p $OUT
for cfg in "--k 44100 --c 1 --dtype f32" "--k 44100 --c 2 --dtype i16" "--k 44100 --c 1 --dtype i16" "--k 20000 --c 1 --dtype f32" \
           "--k 44100 --c 1 --dtype f32 --algo 3" "--k 1000000 --c 1 --dtype f32"; do
  timeout -k 10 180 python -u tools/tune/ab_libs.py abl/libmavg_cur.so abl/libmavg_latea.so \
     $cfg --rounds 6 --steps 10 >> $OUT/ab.log 2>&1 || { echo "ab failed: $cfg"; exit 1; }
  tail -4 $OUT/ab.log | head -3 | cut -c1-120
done
