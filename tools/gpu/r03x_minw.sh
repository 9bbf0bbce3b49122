#!/bin/bash
# look-ahead scan compiled for one more workgroup per CU (launch bounds: fp32 6, int16 7; a few bytes of
# scratch in the record paths) against the release build, in-process A/B
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03x_minw}
mkdir -p $OUT
for cfg in "--k 44100 --c 1 --dtype f32" "--k 44100 --c 2 --dtype i16" "--k 44100 --c 1 --dtype i16" "--k 20000 --c 1 --dtype f32" \
           "--k 1000000 --c 1 --dtype f32"; do
  timeout -k 10 180 python -u tools/tune/ab_libs.py abl/libmavg_cur.so abl/libmavg_minw.so \
     $cfg --rounds 6 --steps 10 >> $OUT/ab.log 2>&1 || { echo "ab failed: $cfg"; exit 1; }
  tail -4 $OUT/ab.log | head -3 | cut -c1-120
done
