#!/bin/bash
# which memory instructions the int16 DMA tile issues at each x[n-k] offset (k = 1016, 1020, 1022, 1023)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/pmc_wr && cd gpurun_out/pmc_wr && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_FLAT SQ_INSTS_VMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_LDS TA_FLAT_WRITE_WAVEFRONTS_sum TA_BUFFER_WRITE_WAVEFRONTS_sum"
for k in 1016 1020 1022 1023; do
  timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d k$k -o run -- ../../tools/tune/tune_scan_nohoist 30 $k 2 i16 1 "i16 tdmw U2 nt13 wg512 dmatrue" > k$k.log 2>&1 || { echo "rc=$? k$k"; exit 1; }
  tail -3 k$k.log
done
