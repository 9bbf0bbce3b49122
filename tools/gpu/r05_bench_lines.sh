#!/bin/bash
# Round 5: one bench.py line per named workload (bench.py's own timing, no CPU
# baseline), e.g.  tools/gpu/r05_bench_lines.sh r05a f32_c8_long f32_c4_long ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:?session tag}
shift
mkdir -p "$OUT"
for w in "$@"; do
  timeout -k 10 150 python -u bench.py --workload "$w" --steps 20 --warmup 5 --no-cpu-baseline \
    > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err"
  rc=$?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], r['frac'], r['frac_of_copy'], r['kernel'])" "$OUT/bench_$w.json" "$w"
  [ $rc -ne 0 ] && { tail -20 "$OUT/bench_$w.err"; exit $rc; }
done
exit 0
