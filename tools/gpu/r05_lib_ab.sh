#!/bin/bash
# Round 5: A/B of the release library against a variant build (make -C
# digital_signal_processsing_amd/csrc variant V=<name> VFLAGS=...) over the
# bench workloads' shapes, with tools/tune/ab_libs.py (outputs compared).
#   tools/gpu/r05_lib_ab.sh <tag> <variant lib> [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:?session tag}
VAR=${2:?variant library}
R=${3:-6}
REL=digital_signal_processsing_amd/lib/libmavg.so
mkdir -p "$OUT"
while read -r name args; do
  [ -z "$name" ] && continue
  timeout -k 10 150 python3 -u tools/tune/ab_libs.py $REL $VAR --rounds "$R" $args > "$OUT/ab_$name.log" 2>&1 \
    || { tail -20 "$OUT/ab_$name.log"; exit 1; }
  echo "== $name"; grep -v amdgpu.ids "$OUT/ab_$name.log" | cut -c1-150
done <<'LIST'
headline --dtype f32 --k 1024 --c 1
i16_2p30 --dtype i16 --k 1024 --c 1
long_2p30 --dtype f32 --k 44100 --c 1
long_1m --dtype f32 --k 1000000 --c 1
long_4m --dtype f32 --k 4000000 --c 1
i16_long --dtype i16 --k 44100 --c 1
i16_stereo_long --dtype i16 --k 44100 --c 2
f32_c4_2p30 --dtype f32 --k 1024 --c 4
f32_c8_2p30 --dtype f32 --k 1024 --c 8
i16_c4_2p30 --dtype i16 --k 1024 --c 4
i16_c8_2p30 --dtype i16 --k 1024 --c 8
f32_c8_long --dtype f32 --k 44100 --c 8
f32_c4_long --dtype f32 --k 44100 --c 4
direct_2p28 --dtype f32 --k 7 --c 1 --log2n 28
LIST
exit 0
