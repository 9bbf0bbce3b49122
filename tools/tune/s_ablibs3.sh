#!/bin/bash
# bench-environment A/B of int16 tile shapes: tuned dispatch (register-staged U4 x 256) vs U2 x 512 (block_size 512)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r02_ablibs3
L=tools/tune/lib_nodma/libmavg.so
for spec in "--k 1024 --c 1" "--k 512 --c 1" "--k 2048 --c 1" "--k 64 --c 1" "--k 1024 --c 2" "--k 300 --c 2"; do
  timeout -k 10 300 python tools/tune/ab_libs.py $L $L --blocks 0 512 $spec --rounds 8 --steps 20 >> gpurun_out/r02_ablibs3/ab.log 2>&1 || exit 1
done
cat gpurun_out/r02_ablibs3/ab.log
