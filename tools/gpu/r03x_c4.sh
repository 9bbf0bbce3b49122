#!/bin/bash
# fp32 4-channel look-ahead scan with 2 frames (32 B) per lane unit: parity, then A/B against the 1-frame units
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03x_c4}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "channel or window_edges or ahead or history or misaligned or unaligned" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for cfg in "--k 2000 --c 4 --dtype f32" "--k 44100 --c 4 --dtype f32" "--k 1001 --c 4 --dtype f32"; do
  timeout -k 10 180 python -u tools/tune/ab_libs.py abl/libmavg_cur.so digital_signal_processsing_amd/lib/libmavg.so \
     $cfg --rounds 6 --steps 10 >> $OUT/ab.log 2>&1 || { echo "ab failed: $cfg"; exit 1; }
  tail -4 $OUT/ab.log | head -3 | cut -c1-150
done
