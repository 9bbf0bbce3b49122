#!/bin/bash
# pmc_pair.sh TAG "name|tune_scan args" ... : the pmc_long.sh counter groups
# (A, B, C) for arbitrary tune_scan variants, each group in its own
# rocprofv3 pass; tabulate with tools/pmc_table.py gpurun_out/TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
mkdir -p gpurun_out/$TAG && cd gpurun_out/$TAG && export TMPDIR=/tmp
T=../../tools/tune/${BIN:-tune_scan}
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
B="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA"
C="SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum"
for w in "$@"; do
  tag=${w%%|*}; spec=${w#*|}
  for g in A B C; do
    eval "set -- $spec"
    timeout -s KILL 90 rocprofv3 --pmc ${!g} --output-format csv -d ${tag}_$g -o run -- $T "$@" > ${tag}_$g.log 2>&1 \
      || { echo "rc=$? ${tag}_$g"; exit 1; }
  done
done
echo done
