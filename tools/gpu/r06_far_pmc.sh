#!/bin/bash
# Round 6: memory-side counters of the very-long-window look-ahead forms (tools/tune/wide_ab "self"
# mode, fp32 mono): one variant per process (WIDE_AB_ONLY), each counter group in its own
# rocprofv3 --pmc pass under its own limit:
#   FETCH_SIZE | WRITE_SIZE | TCC_EA0_RDREQ_sum + TCC_EA0_RDREQ_DRAM_sum |
#   TCC_EA0_RDREQ_32B_sum + TCC_EA0_RDREQ_64B_sum + TCC_EA0_RDREQ_128B_sum
#   tools/gpu/r06_far_pmc.sh <tag> <variant regex> <k> [<k> ...]
# then: python3 tools/tune/pmc_far.py gpurun_out/<tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:?session tag}
RX=${2:?variant regex}
shift 2
mkdir -p "$OUT"
GROUPS_=("FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"
         "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum")
for k in "$@"; do
  WIDE_AB_LIST=1 timeout -k 10 60 tools/tune/wide_ab 30 "$k" 1 1 0 f32 self > "$OUT/k${k}_variants.tsv" || exit 1
  grep -E "$RX" "$OUT/k${k}_variants.tsv" > "$OUT/k${k}_selected.tsv"
  while IFS=$'\t' read -r i name; do
    g=0
    for grp in "${GROUPS_[@]}"; do
      WIDE_AB_ONLY=$i timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv \
        -d "$OUT/k${k}_v${i}_g${g}" -o pmc -- tools/tune/wide_ab 30 "$k" 1 1 0 f32 self \
        > "$OUT/k${k}_v${i}_g${g}.log" 2>&1 || { tail -20 "$OUT/k${k}_v${i}_g${g}.log"; exit 1; }
      g=$((g + 1))
    done
    echo "k=$k variant $i ($name) done"
  done < "$OUT/k${k}_selected.tsv"
done
exit 0
