#!/bin/bash
# Round 6: the wave scans' DPP moves with bound_ctrl zero fill (no destination zero init on the
# row_shr steps) and the Hillis-Steele log-step scans interleaved (wave_incl_scan_n), against the
# release library, in bench.py's environment (tools/tune/ab_libs.py).
#   tools/gpu/r06_dpp_ab.sh <tag> <lib> [<lib> ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:?session tag}; shift
mkdir -p $O
R=digital_signal_processsing_amd/lib/libmavg.so
ab() { n=$1; shift; timeout -k 10 200 python3 -u tools/tune/ab_libs.py $R "${LIBS[@]}" --rounds 6 "$@" > $O/ab_$n.log 2>&1 || return 1
       echo "== $n"; grep -v amdgpu.ids $O/ab_$n.log | cut -c1-150; }
LIBS=("$@")
ab hillis_long --dtype f32 --k 44100 --c 1 --algo 3 && ab hillis_2p30 --dtype f32 --k 1024 --c 1 --algo 3 && \
ab hillis_i16_long --dtype i16 --k 44100 --c 1 --algo 3 && ab hillis_i16_2p30 --dtype i16 --k 1024 --c 1 --algo 3 && \
ab hillis_i16_stereo --dtype i16 --k 44100 --c 2 --algo 3 && \
ab headline --dtype f32 --k 1024 --c 1 && ab long_2p30 --dtype f32 --k 44100 --c 1 && \
ab f32_c8_long --dtype f32 --k 44100 --c 8 && ab i16_c8_2p30 --dtype i16 --k 1024 --c 8 && \
ab f32_c4_long --dtype f32 --k 44100 --c 4 && ab i16_long --dtype i16 --k 44100 --c 1
