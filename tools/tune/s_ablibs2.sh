#!/bin/bash
# bench-environment A/B of the fp32 LDS-DMA tile rule (headline and configs #2 / #4 windows)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r02_ablibs2
A=tools/tune/lib_nodma/libmavg.so; B=tools/tune/lib_nof32dma/libmavg.so
for spec in "--k 1024" "--k 4096" "--k 64" "--k 1023" "--k 1024"; do
  timeout -k 10 300 python tools/tune/ab_libs.py $A $B $spec --dtype f32 --rounds 8 --steps 20 >> gpurun_out/r02_ablibs2/ab.log 2>&1 || exit 1
done
cat gpurun_out/r02_ablibs2/ab.log
