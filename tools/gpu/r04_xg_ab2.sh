#!/bin/bash
# Round 4: the halo-only chan tile past 32 KiB of halo (release) against the
# previous dispatch (lib/libmavg_noxg.so, -DMAVG_NO_CHAN_XG), bench.py's timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r04_xg_ab2}
mkdir -p "$OUT"
L=digital_signal_processsing_amd/lib
for spec in "1536 8" "2048 8" "2048 4" "3000 4"; do
  read -r k c <<< "$spec"
  timeout -k 10 200 python -u tools/tune/ab_libs.py $L/libmavg_noxg.so $L/libmavg.so --k "$k" --c "$c" \
    --dtype f32 --dist 2 --rounds 8 > "$OUT/bench_timing_xg_c${c}_k${k}.log" 2>&1
  rc=$?
  cat "$OUT/bench_timing_xg_c${c}_k${k}.log"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
