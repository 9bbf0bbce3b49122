#!/bin/bash
# PMC comparison of the long-window look-ahead scan (fp32 mono, int16 stereo,
# int16 stereo with the look-ahead work switched off) against the int16 stereo
# tile scan at k=1024; each counter group in its own rocprofv3 pass.
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
for w in "f32ahead|30 44100 2 f32 1 \"ahead U4 pf4\"" "i16sahead|30 44100 2 i16 1 \"stereo ahead tile-records pf1\" 2" \
         "i16sdbg7|30 44100 2 i16 1 \"stereo ahead dbg7\" 2" "i16stile|30 1024 2 i16 1 \"stereo tileS U4 nt3 wg256\" 2" \
         ${EXTRA:-}; do
  tag=${w%%|*}; spec=${w#*|}
  for g in A B C; do PMC=${!g} pass ${tag}_$g "$spec" || exit 1; done
done
echo done
