#!/bin/bash
# self-published records: consumer polls (MAVG_AHEAD_STATS builds, look-ahead vs self) at 8192 / 20000 / 44100,
# and the release build against forced self-publication for fp32 stereo and the Hillis-Steele flavour
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03x_self3}
mkdir -p $OUT
for k in 8192 20000 44100; do
  timeout -k 10 120 python -u tools/tune/ahead_stats.py abl/libmavg_stats.so abl/libmavg_stats_self.so --k $k >> $OUT/stats.log 2>&1 \
    || { echo "stats failed: $k"; exit 1; }
done
grep -v amdgpu.ids $OUT/stats.log | cut -c1-160
for cfg in "--k 3000 --c 2 --dtype f32" "--k 6000 --c 2 --dtype f32" "--k 5000 --c 1 --dtype f32 --algo 3" "--k 8192 --c 1 --dtype f32 --algo 3" \
           "--k 12288 --c 1 --dtype f32 --algo 3"; do
  timeout -k 10 180 python -u tools/tune/ab_libs.py abl/libmavg_cur.so abl/libmavg_self.so \
     $cfg --rounds 6 --steps 10 >> $OUT/ab.log 2>&1 || { echo "ab failed: $cfg"; exit 1; }
  tail -4 $OUT/ab.log | head -3 | cut -c1-120
done
