#!/bin/bash
# write-through (sc1) output stores (abl/libmavg_wt.so: -DMAVG_AHEAD_WT_STORE=1 -DMAVG_TILE_WT_STORE=1) against
# the release build (plain / nt stores keep the output lines in the XCD L2), in-process A/B. The variant
# (buffer_store_dwordx4 sc1 through a per-tile descriptor) was measured slower and not kept.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03x_wt}
mkdir -p $OUT
for cfg in "--k 44100 --c 1 --dtype f32" "--k 44100 --c 2 --dtype i16" "--k 44100 --c 1 --dtype i16" "--k 4000000 --c 1 --dtype f32" \
           "--k 1000000 --c 1 --dtype f32" "--k 1024 --c 1 --dtype f32" "--k 4096 --c 1 --dtype f32" "--k 1024 --c 2 --dtype i16" \
           "--k 64 --c 1 --dtype f32 --log2n 26"; do
  timeout -k 10 180 python -u tools/tune/ab_libs.py abl/libmavg_cur.so abl/libmavg_wt.so \
     $cfg --rounds 6 --steps 10 >> $OUT/ab.log 2>&1 || { echo "ab failed: $cfg"; exit 1; }
  tail -4 $OUT/ab.log | head -3 | cut -c1-120
done
