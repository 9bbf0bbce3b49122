#!/bin/bash
# Round 5: HBM traffic of each very-long-window footprint variant of the tuner
# (tools/tune/wide_ab, mono fp32: look-ahead distance D and the 2-workgroups-
# per-CU cap) -- one variant per process (WIDE_AB_ONLY), FETCH_SIZE and
# WRITE_SIZE in separate rocprofv3 --pmc passes, each pass under its own limit.
#   tools/gpu/r05_footprint_pmc.sh <tag> <k> [<k> ...]
# then: python3 tools/tune/pmc_variants.py gpurun_out/<tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:?session tag}
shift
mkdir -p "$OUT"
for k in "$@"; do
  WIDE_AB_LIST=1 timeout -k 10 60 tools/tune/wide_ab 30 "$k" 1 1 2 > "$OUT/k${k}_variants.tsv" || exit 1
  while IFS=$'\t' read -r i name; do
    for c in FETCH_SIZE WRITE_SIZE; do
      WIDE_AB_ONLY=$i timeout -s KILL 90 rocprofv3 --pmc "$c" --output-format csv \
        -d "$OUT/k${k}_v${i}_${c}" -o pmc -- tools/tune/wide_ab 30 "$k" 1 1 2 \
        > "$OUT/k${k}_v${i}_${c}.log" 2>&1 || { tail -20 "$OUT/k${k}_v${i}_${c}.log"; exit 1; }
    done
    echo "k=$k variant $i ($name) done"
  done < "$OUT/k${k}_variants.tsv"
done
exit 0
