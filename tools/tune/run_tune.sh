#!/bin/bash
# run_tune.sh TAG "lg k rounds dtype burst filter channels" ... : several tune_scan runs, each under its own time limit
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
for spec in "$@"; do
  i=$((i+1))
  eval "set -- $spec"
  timeout -k 10 150 tools/tune/${BIN:-tune_scan} "$@" > $OUT/run$i.log 2>&1; rc=$?
  echo "== run$i: $spec (rc=$rc)"; grep -v "recomputes" $OUT/run$i.log | tail -n +3
  [ $rc -ne 0 ] && { echo "FATAL rc=$rc"; exit $rc; }
done
echo tune done
