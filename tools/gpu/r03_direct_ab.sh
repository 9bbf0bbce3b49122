#!/bin/bash
# config #3 direct-kernel shape, one interleaved A/B per box:
# round-1 shape (U=1, default policy) vs the round-2 shape (U=2, nt=11), 2^28 fp32, k=7
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-direct_ab}
mkdir -p $OUT
timeout -k 10 120 python -u tools/tune/ab_libs.py abl/libmavg_direct_r1.so digital_signal_processsing_amd/lib/libmavg.so \
  --algo 5 --k 7 --c 1 --dtype f32 --log2n 28 --rounds 16 --steps 10 > $OUT/direct_ab.log 2>&1
rc=$?; echo "direct A/B rc=$rc (box $(hostname))"; cat $OUT/direct_ab.log | cut -c1-170; exit $rc
