#!/bin/bash
# Round 4: the wide-frame tile scan's shapes against the library's dispatch
# (tools/tune/wide_ab), fp32 C = 2, 4, 8, then the GPU test suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r04_wide}
mkdir -p "$OUT"
shift || true
for spec in "$@"; do
  IFS=: read -r k C <<< "$spec"
  echo "== wide_ab k=$k C=$C"
  IFS=: read -r k C DT <<< "$spec"; DT=${DT:-f32}
  timeout -k 10 150 tools/tune/wide_ab 30 "$k" "$C" 6 1 "$DT" > "$OUT/${DT}_c${C}_k${k}.log" 2>&1
  rc=$?
  cat "$OUT/${DT}_c${C}_k${k}.log"
  [ $rc -ne 0 ] && { echo "wide_ab rc=$rc: stopping"; exit $rc; }
done
exit 0
