#!/bin/bash
# PMC comparison of the long-window look-ahead scan (the bench's fp32 mono,
# int16 mono and int16 stereo shapes at k=44100) against the tile scans at
# k=1024; each counter group in its own rocprofv3 pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-pmc_long}
mkdir -p gpurun_out/$TAG && cd gpurun_out/$TAG && export TMPDIR=/tmp
T=../../tools/tune/tune_scan
pass() { local tag=$1 spec=$2; shift 2
  eval "set -- $spec \"\$@\""
  local args=("$@")
  timeout -s KILL 90 rocprofv3 --pmc ${PMC} --output-format csv -d $tag -o run -- $T "${args[@]}" > $tag.log 2>&1 || { echo "rc=$? $tag"; exit 1; }; }
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
B="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA"
C="SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum"
for w in "f32ahead|30 44100 2 f32 1 \"ahead U4 rctrue dmatrue D512 wtrue nt9\"" \
         "i16ahead|30 44100 2 i16 1 \"i16 ahead U4 rcfalse dmatrue D512 wtrue nt9\" 1" \
         "i16sahead|30 44100 2 i16 1 \"stereo ahead U4 rcfalse dmatrue D768 wfalse nt9\" 2" \
         "i16stile|30 1024 2 i16 1 \"stereo tile U4 nt3 div1\" 2" "f32tile|30 1024 2 f32 1 \"tileS U2 nt13 wg256\"" \
         ${EXTRA:-}; do
  tag=${w%%|*}; spec=${w#*|}
  for g in A B C; do PMC=${!g} pass ${tag}_$g "$spec" || exit 1; done
done
echo done
