mkdir -p gpurun_out/pmc2 && cd gpurun_out/pmc2 && export TMPDIR=/tmp
rocprofv3 -L > counters.txt 2>&1 || true
T=../../tools/tune/tune_scan
F="copy flat|tile U2 remap64"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d p1 -o run -- $T 30 1024 2 f32 1 "$F" > p1.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d p2 -o run -- $T 30 1024 2 f32 1 "$F" > p2.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU --output-format csv -d p3 -o run -- $T 30 1024 2 f32 1 "$F" > p3.log 2>&1
echo done
