#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/kscan; mkdir -p $OUT
for k in 65535 65536 100000 441000; do
  for C in 1 2; do
    timeout -k 10 120 tools/tune/tune_scan 30 $k 4 i16 10 "copy flat|product" $C > $OUT/i16_C${C}_k$k.log 2>&1 || { echo "rc=$? i16 k=$k C=$C"; exit 1; }
  done
done
for k in 100000 200000 1000000; do
  timeout -k 10 120 tools/tune/tune_scan 30 $k 4 f32 10 "copy flat|product" > $OUT/f32_k$k.log 2>&1 || { echo "rc=$? f32 k=$k"; exit 1; }
done
echo done
