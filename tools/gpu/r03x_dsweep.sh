#!/bin/bash
# look-ahead distance D per window length (tools/tune/d_sweep.py), in one process per config
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03x_dsweep}
mkdir -p $OUT
run() { timeout -k 10 240 python -u tools/tune/d_sweep.py "$@" >> $OUT/dsweep.log 2>&1 || { echo "sweep failed: $*"; exit 1; }
        tail -8 $OUT/dsweep.log | grep -E "^(n=|D=)" | cut -c1-80; }
run --k 4000000 --c 1 --dtype f32 --slots 1024 1536 2048 3072 4096
run --k 2000000 --c 1 --dtype f32 --slots 1024 1536 2048 3072
run --k 1000000 --c 1 --dtype f32 --slots 512 1024 1536 2048
run --k 1000000 --c 2 --dtype i16 --slots 768 1024 1536 2048
run --k 1500000 --c 1 --dtype i16 --slots 1024 1536 2048
