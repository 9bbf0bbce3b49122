#!/bin/bash
# does the int16 DMA tile's speed depend on where y sits relative to x? (bench.py buffers vs the tuner's)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r02_ypad
A=tools/tune/lib_dma/libmavg.so; B=tools/tune/lib_nodma/libmavg.so
for pad in 0 4096 65536 1048576 33554432; do
  timeout -k 10 300 python tools/tune/ab_libs.py $A $B --k 1024 --c 1 --ypad $pad --rounds 6 --steps 20 >> gpurun_out/r02_ypad/ab.log 2>&1 || exit 1
done
timeout -k 10 200 tools/tune/tune_scan 30 1024 8 i16 -20 "copy flat|i16 tdmw U2 nt13 wg512 dmatrue|i16 tdma U4 nt3 dmafalse" >> gpurun_out/r02_ypad/ab.log 2>&1
grep -v "torch copy\|amdgpu.ids" gpurun_out/r02_ypad/ab.log | cut -c1-150
