#!/bin/bash
# channel-count survey of the release build (the library timed twice, interleaved): fp32 and int16 at C = 1, 2, 4, 8 (2^30 divisible by C)
# at k=1024 and k=44100, 2^30 samples; for DESIGN's multi-channel notes
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03y_channels}
mkdir -p $OUT
L=digital_signal_processsing_amd/lib/libmavg.so
for dt in f32 i16; do
  for c in 1 2 4 8; do
    for k in 1024 44100; do
      timeout -k 10 120 python -u tools/tune/ab_libs.py $L $L --k $k --c $c --dtype $dt --rounds 2 --steps 5 >> $OUT/survey.log 2>&1 \
        || { echo "survey failed: $dt $c $k"; exit 1; }
      echo "$dt C=$c k=$k $(tail -3 $OUT/survey.log | head -1 | grep -o 'mean [0-9.]* ms ([0-9.]* of 8 TB/s)')"
    done
  done
done
