#!/bin/bash
# fp32 8-channel Blelloch path in 64-B units (2 frames per lane) against the 1-frame units: parity, then A/B
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03y_c8}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "channel or window_edges or misaligned or unaligned or golden or block" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for k in 7 1024 44100; do
  timeout -k 10 180 python -u tools/tune/ab_libs.py abl/libmavg_cur.so digital_signal_processsing_amd/lib/libmavg.so \
     --k $k --c 8 --dtype f32 --rounds 4 --steps 10 >> $OUT/ab.log 2>&1 || { echo "ab failed: $k"; exit 1; }
  tail -4 $OUT/ab.log | head -3 | cut -c1-150
done
