#!/bin/bash
# self-published records beyond fp32 mono (abl/libmavg_self.so, -DMAVG_AHEAD_SELF=1 forces them):
# fp32 stereo / 4 channels and the Hillis-Steele flavour at windows of <= 3 tiles, against the release build
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03x_self4}
mkdir -p $OUT
for cfg in "--k 3000 --c 2 --dtype f32" "--k 6000 --c 2 --dtype f32" "--k 2000 --c 4 --dtype f32" \
           "--k 5000 --c 1 --dtype f32 --algo 3" "--k 8192 --c 1 --dtype f32 --algo 3" "--k 12288 --c 1 --dtype f32 --algo 3" \
           "--k 8192 --c 1 --dtype f32"; do
  timeout -k 10 180 python -u tools/tune/ab_libs.py abl/libmavg_cur.so abl/libmavg_self.so \
     $cfg --rounds 6 --steps 10 >> $OUT/ab.log 2>&1 || { echo "ab failed: $cfg"; exit 1; }
  tail -4 $OUT/ab.log | head -3 | cut -c1-150
done
