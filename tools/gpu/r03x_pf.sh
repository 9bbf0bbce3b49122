#!/bin/bash
# self-published records with an L2 touch of the tile D slots ahead (abl/libmavg_pf.so, -DMAVG_AHEAD_SELF=2:
# no phase A, one 4-B load per 128-B line of tile t+D never waited for) against the release build.
# Measured slower everywhere and not kept (look-ahead scan item 5).
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03x_pf}
mkdir -p $OUT
for cfg in "--k 44100 --c 1 --dtype f32" "--k 20000 --c 1 --dtype f32" "--k 44100 --c 2 --dtype i16" "--k 44100 --c 1 --dtype i16" \
           "--k 8192 --c 1 --dtype f32" "--k 44100 --c 1 --dtype f32 --algo 3" "--k 1000000 --c 1 --dtype f32"; do
  timeout -k 10 180 python -u tools/tune/ab_libs.py abl/libmavg_cur.so abl/libmavg_pf.so \
     $cfg --rounds 6 --steps 10 >> $OUT/ab.log 2>&1 || { echo "ab failed: $cfg"; exit 1; }
  tail -4 $OUT/ab.log | head -3 | cut -c1-120
done
