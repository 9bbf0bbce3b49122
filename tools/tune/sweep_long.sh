#!/bin/bash
# Long windows (look-ahead scan) at 2^30: fp32 mono, int16 mono, int16 stereo, against the flat copy.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-sweep_long}; mkdir -p $OUT
run() { local tag=$1; shift; timeout -k 10 150 tools/tune/tune_scan "$@" > $OUT/$tag.log 2>&1; local rc=$?; [ $rc -ge 124 ] && { echo "FATAL $rc in $tag"; exit $rc; }; [ $rc -ne 0 ] && echo "rc=$rc in $tag"; tail -12 $OUT/$tag.log; return 0; }
F=${FILTER:-copy flat|ahead|product}
for k in ${KS:-44100}; do
  run f32_k$k 30 $k 6 f32 10 "$F" || exit 1
  run i16C1_k$k 30 $k 6 i16 10 "$F" 1 || exit 1
  run i16C2_k$k 30 $k 6 i16 10 "$F" 2 || exit 1
done
echo sweep done
