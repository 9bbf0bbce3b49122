#!/bin/bash
# Round 6: the release library against a variant build (make -C digital_signal_processsing_amd/csrc
# variant V=<name> VFLAGS=...) at named shapes, in bench.py's environment (tools/tune/ab_libs.py:
# torch buffers, one HIP-event pair per launch, outputs compared).
#   tools/gpu/r06_lib_ab.sh <tag> <variant lib> <rounds> <name>:<dtype>:<k>:<C> [...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:?session tag}
VAR=${2:?variant library}
R=${3:?rounds}
shift 3
REL=digital_signal_processsing_amd/lib/libmavg.so
mkdir -p "$OUT"
for s in "$@"; do
  IFS=: read -r name dt k c <<< "$s"
  timeout -k 10 200 python3 -u tools/tune/ab_libs.py $REL $VAR --rounds "$R" --dtype "$dt" --k "$k" --c "$c" \
    > "$OUT/ab_$name.log" 2>&1 || { tail -20 "$OUT/ab_$name.log"; exit 1; }
  echo "== $name"; grep -v amdgpu.ids "$OUT/ab_$name.log" | cut -c1-150
done
exit 0
