#!/bin/bash
# PMC comparison: int16 mono tile scan (k=1024) vs look-ahead scan (k=44100),
# each counter group in its own rocprofv3 pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc_ahead && cd gpurun_out/pmc_ahead && export TMPDIR=/tmp
T=../../tools/tune/tune_scan
pass() { local tag=$1 k=$2 filt=$3; shift 3
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $tag -o run -- $T 30 $k 2 i16 1 "$filt" 1 > $tag.log 2>&1 || { echo "rc=$? $tag"; exit 1; }; }
for w in "tile 1024 product" "ahead 44100 i16 ahead U4"; do
  set -- $w; tag=$1; k=$2; shift 2; filt="$*"
  pass ${tag}_a $k "$filt" SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
  pass ${tag}_b $k "$filt" SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM
  pass ${tag}_c $k "$filt" TCC_HIT_sum TCC_MISS_sum
done
echo done
