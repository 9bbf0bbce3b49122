#!/bin/bash
# bench-environment A/B of the int16 LDS-DMA tile rule: the product library against a build without it
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r02_ablibs
A=digital_signal_processsing_amd/lib/libmavg.so; B=tools/tune/lib_nodma/libmavg.so
for spec in "--k 1024 --c 1" "--k 1024 --c 2" "--k 512 --c 1" "--k 2048 --c 1"; do
  timeout -k 10 300 python tools/tune/ab_libs.py $A $B $spec --rounds 8 --steps 20 >> gpurun_out/r02_ablibs/ab.log 2>&1 || exit 1
done
cat gpurun_out/r02_ablibs/ab.log
