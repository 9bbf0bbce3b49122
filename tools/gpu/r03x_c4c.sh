#!/bin/bash
# fp32 4-channel shapes as dispatched (32-B units: 1024-frame tiles up to 4 KiB of halo, then the
# look-ahead scan in 1024-frame tiles): parity, then A/B against the 1-frame units (abl/libmavg_cur.so)
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03x_c4c}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "four_channels or channel or window_edges or ahead or history or misaligned or unaligned or golden or ragged or block" \
  > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for k in 7 257 500 1001 2000 44100; do
  timeout -k 10 180 python -u tools/tune/ab_libs.py abl/libmavg_cur.so digital_signal_processsing_amd/lib/libmavg.so \
     --k $k --c 4 --dtype f32 --rounds 4 --steps 10 >> $OUT/ab.log 2>&1 || { echo "ab failed: $k"; exit 1; }
  tail -4 $OUT/ab.log | head -3 | cut -c1-150
done
