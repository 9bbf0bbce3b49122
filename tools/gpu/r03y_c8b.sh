#!/bin/bash
# final tree: full GPU suite and smoke, then the fp32 8-channel A/B as dispatched (64-B units past k=256)
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03y_c8b}
mkdir -p $OUT
bash tools/gpu_session.sh ${1:-r03y_c8b} testx smoke || exit $?
grep -q "FATAL" $OUT/session.log && exit 1
grep -q "pytest_gpu rc=0" $OUT/session.log || exit 1
for k in 7 300 1024 44100; do
  timeout -k 10 180 python -u tools/tune/ab_libs.py abl/libmavg_cur.so digital_signal_processsing_amd/lib/libmavg.so \
     --k $k --c 8 --dtype f32 --rounds 4 --steps 10 >> $OUT/ab.log 2>&1 || { echo "ab failed: $k"; exit 1; }
  tail -4 $OUT/ab.log | head -3 | cut -c1-150
done
