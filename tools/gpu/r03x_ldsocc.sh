#!/bin/bash
# look-ahead scan occupancy lowered through the LDS allocation (32 KiB: 5 workgroups per CU, 40 KiB: 4)
# against the release build, in-process A/B
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03x_ldsocc}
mkdir -p $OUT
for cfg in "--k 44100 --c 1 --dtype f32" "--k 44100 --c 2 --dtype i16" "--k 44100 --c 1 --dtype i16" "--k 20000 --c 1 --dtype f32" \
           "--k 1000000 --c 1 --dtype f32"; do
  timeout -k 10 180 python -u tools/tune/ab_libs.py abl/libmavg_cur.so abl/libmavg_lds32768.so abl/libmavg_lds40960.so \
     $cfg --rounds 6 --steps 10 >> $OUT/ab.log 2>&1 || { echo "ab failed: $cfg"; exit 1; }
  tail -5 $OUT/ab.log | head -4 | cut -c1-120
done
