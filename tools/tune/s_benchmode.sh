#!/bin/bash
# the tuner in bench.py's timing mode (burst -20): does it rank the int16 / fp32 tile shapes as ab_libs.py did?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
M='"copy flat|i16 tdmw U2 nt13 wg512 dmatrue|i16 tdma U4 nt3 dmafalse|i16 tdmw U2 nt3 wg512 dmafalse|i16 product"'
S='"copy flat|i16 stereo tdma U8 nt13 dmatrue|i16 stereo tdma U4 nt3 dmafalse|stereo product"'
F='"copy flat|tdma U2 nt13 wg512 dmatrue|tdma U2 nt13 wg512 dmafalse|tdma U2 nt13 wg256 dmafalse|f32 product"'
tools/tune/run_tune.sh r02_benchmode "30 1024 8 i16 -20 $M" "30 1024 8 i16 -20 $S 2" "30 1024 6 f32 -20 $F" "30 64 6 f32 -20 $F" \
  "30 1024 8 i16 10 $M" "30 1024 6 f32 10 $F"
