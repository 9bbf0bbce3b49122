#!/bin/bash
# small look-ahead distances down to D = 0 (every tile publishes its own record, phase A re-reads it)
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03x_dsmall}
mkdir -p $OUT
run() { timeout -k 10 240 python -u tools/tune/d_sweep.py "$@" >> $OUT/dsweep.log 2>&1 || { echo "sweep failed: $*"; exit 1; }
        tail -8 $OUT/dsweep.log | grep -E "^(n=|D=)" | cut -c1-80; }
run --k 44100 --c 1 --dtype f32 --slots 0 8 64 128 256 512
run --k 44100 --c 2 --dtype i16 --slots 0 8 64 256 768
run --k 44100 --c 1 --dtype i16 --slots 0 8 64 256 512
run --k 1000000 --c 1 --dtype f32 --slots 0 64 256 1024
