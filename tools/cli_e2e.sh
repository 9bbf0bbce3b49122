#!/bin/bash
# End-to-end (PCIe-inclusive) CLI numbers on a large stereo WAV: the reference's
# own timing model (H2D + kernel + D2H) with pageable host buffers; page-locking
# them (hipHostRegister) measured no faster: 56 GB/s either way.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/cli_e2e; mkdir -p $OUT
python -c "
import sys; sys.path.insert(0,'digital_signal_processsing_amd/cli')
import run_benchmarks as rb; rb.generate_wav(50_000_000, path='$OUT/big.wav', seed=1)"
cd $OUT
B=../../digital_signal_processsing_amd/cli
for bin in bin_vblelloch bin_vec4 bin_vhillis; do
  timeout -k 10 300 $B/$bin big.wav 1024 256 > $bin.log 2>&1 || exit $?
done
timeout -k 10 300 $B/bin_cpu big.wav 1024 256 > bin_cpu.log 2>&1
rm -f big.wav
echo done
