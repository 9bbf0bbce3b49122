#!/bin/bash
# Round 6: the release library against a variant build over the windows past the L2 reach, in
# bench.py's environment (tools/tune/ab_libs.py: torch buffers, one HIP-event pair per launch,
# outputs compared), because the in-process tuner and bench.py's timing disagreed there.
#   tools/gpu/r06_far_ab.sh <tag> <variant lib> [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:?session tag}
VAR=${2:?variant library}
R=${3:-6}
REL=digital_signal_processsing_amd/lib/libmavg.so
mkdir -p "$OUT"
while read -r name args; do
  [ -z "$name" ] && continue
  timeout -k 10 200 python3 -u tools/tune/ab_libs.py $REL $VAR --rounds "$R" $args > "$OUT/ab_$name.log" 2>&1 \
    || { tail -20 "$OUT/ab_$name.log"; exit 1; }
  echo "== $name"; grep -v amdgpu.ids "$OUT/ab_$name.log" | cut -c1-150
done <<'LIST'
long_1m --dtype f32 --k 1000000 --c 1
long_2m --dtype f32 --k 2000000 --c 1
long_4m --dtype f32 --k 4000000 --c 1
f32_6e5 --dtype f32 --k 600000 --c 1
i16_stereo_2m --dtype i16 --k 2000000 --c 2
i16_stereo_6e5 --dtype i16 --k 600000 --c 2
i16_mono_1m5 --dtype i16 --k 1500000 --c 1
LIST
exit 0
