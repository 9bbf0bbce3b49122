#!/bin/bash
# int16 windows not a multiple of the lane unit, after the whole-unit extraction fix; then the GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
M='"copy flat|i16 tdmw U2 nt3 wg256 dmafalse|i16 tdma U4 nt3 dmafalse|i16 tdmw U2 nt13 wg512 dmatrue"'
S='"copy flat|i16 stereo tdma U4 nt3 dmafalse|i16 stereo tdma U8 nt13 dmatrue|i16 stereo tdmw U2 nt3 wg256 dmafalse"'
L='"copy flat|i16 ahead U4 rcfalse dmatrue D512 wtrue nt9|i16 product"'
tools/tune/run_tune.sh r02_odd3 "30 1023 16 i16 10 $M" "30 1020 16 i16 10 $M" "30 7 16 i16 10 $M" "30 12 16 i16 10 $M" \
  "30 1024 16 i16 10 $M" "30 1023 16 i16 10 $S 2" "30 65 16 i16 10 $S 2" "30 44100 8 i16 10 $L" "30 44101 8 i16 10 $L" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r02_odd3/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r02_odd3/pytest_gpu.log; exit $rc
