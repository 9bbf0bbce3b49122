#!/bin/bash
# int16 tile-shape sweep (mono and stereo) over window sizes: the data behind
# dispatch_scan_f's int16 rules.  Run on the GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/sweep_i16; mkdir -p $OUT
for C in 1 2; do
  for k in 64 512 1024 2048 4096 8192; do
    timeout -k 10 120 tools/tune/tune_scan 30 $k 8 i16 10 "copy flat|tile|product" $C > $OUT/C${C}_k${k}.log 2>&1 || exit $?
  done
done
echo sweep done
