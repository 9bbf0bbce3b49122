#!/bin/bash
# look-ahead scan workgroup size, in-process A/B: HEAD build, 256 threads x U=4 (this tree), 512 threads x U=2
# (abl/ libraries built from tuning flags -DMAVG_AHEAD_WG=512; same 4096-frame tiles and records)
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03x_wg}
mkdir -p $OUT
for cfg in "--k 44100 --c 1 --dtype f32 --algo 0" "--k 44100 --c 1 --dtype f32 --algo 3" "--k 44100 --c 2 --dtype i16 --algo 0" \
           "--k 44100 --c 1 --dtype i16 --algo 0" "--k 1000000 --c 1 --dtype f32 --algo 0"; do
  timeout -k 10 180 python -u tools/tune/ab_libs.py abl/libmavg_base.so abl/libmavg_wg256.so abl/libmavg_wg512.so \
     $cfg --rounds 4 --steps 10 >> $OUT/ab.log 2>&1 || { echo "ab failed: $cfg"; exit 1; }
  tail -5 $OUT/ab.log | head -4 | cut -c1-120
done
