#!/bin/bash
# Hillis-Steele look-ahead forms, in-process A/B: HEAD (tile staged in LDS, scan before the carry),
# transposed global tile loads with the scan before (early) or after (late) the carry.
# The two variant libraries were built from a form of mavg_lookback.hpp that was measured slower and
# not kept (Hillis-Steele flavour); the script is the record of the measurement.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03x_hs3}
mkdir -p $OUT
for cfg in "--k 44100 --c 1 --dtype f32" "--k 44100 --c 2 --dtype i16" "--k 44100 --c 1 --dtype i16"; do
  timeout -k 10 180 python -u tools/tune/ab_libs.py abl/libmavg_base.so abl/libmavg_hs_early.so abl/libmavg_hs_late.so \
     $cfg --algo 3 --rounds 4 --steps 10 >> $OUT/ab.log 2>&1 || { echo "ab failed: $cfg"; exit 1; }
  tail -5 $OUT/ab.log | head -4 | cut -c1-120
done
