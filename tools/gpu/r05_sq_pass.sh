#!/bin/bash
# Round 5: one rocprofv3 SQ counter pass per bench workload (wave-cycle split:
# active VALU / LDS / any, waiting, issue-stalled), each under its own limit.
#   tools/gpu/r05_sq_pass.sh <tag> <workload> [<workload> ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:?session tag}
shift
mkdir -p "$OUT"
rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
for w in "$@"; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU \
    --output-format csv -d "$OUT/sq_$w" -o pmc -- python3 bench.py --workload "$w" --steps 10 --warmup 3 --no-cpu-baseline \
    > "$OUT/sq_$w.log" 2>&1 || { tail -20 "$OUT/sq_$w.log"; exit 1; }
  echo "$w done"
done
exit 0
