#!/bin/bash
# Round 4: per-tile phase A loads non-temporal (tools/tune/wide_ab_nta, its
# look-ahead variants) against the release library (the "lib" line), very
# long fp32 windows.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r04_nta}
mkdir -p "$OUT"
for k in 4000000 2000000 44100; do
  timeout -k 10 150 tools/tune/wide_ab_nta 30 "$k" 1 6 1 f32 > "$OUT/nta_k$k.log" 2>&1
  rc=$?
  cat "$OUT/nta_k$k.log"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
