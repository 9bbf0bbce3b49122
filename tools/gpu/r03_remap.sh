#!/bin/bash
# very long windows: round-2 library vs grouped remap (no group records) vs grouped remap + group records
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-r03k}
mkdir -p $OUT
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "ahead or unaligned_and_large or int64_division" > $OUT/pytest_long.log 2>&1
echo "pytest rc=$?"; tail -2 $OUT/pytest_long.log
for cfg in "--k 1000000 --c 1 --dtype f32" "--k 4000000 --c 1 --dtype f32" "--k 1000000 --c 2 --dtype i16" "--k 600000 --c 1 --dtype f32"; do
  for pair in "abl/libmavg_ahead.so abl/libmavg_g64_nogroups.so" "abl/libmavg_g64_nogroups.so digital_signal_processsing_amd/lib/libmavg.so"; do
    $T 180 python -u tools/tune/ab_libs.py $pair $cfg --rounds 4 --steps 10 >> $OUT/ab.log 2>&1 || { echo "ab failed: $cfg"; exit 1; }
    tail -4 $OUT/ab.log | head -3 | cut -c1-120
  done
done
