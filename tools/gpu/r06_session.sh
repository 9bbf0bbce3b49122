#!/bin/bash
# Round 6: one GPU session of named steps, each under its own time limit; the
# first step that fails (non-zero, abort, segfault, time limit) ends the session.
#   tools/gpu/r06_session.sh <tag> <step> [<step> ...]
# steps: counters fullsize_new gloo2 ab_i16_mono ab_i16_stereo ab_i16_c4 ab_i16_c8
#        gpu_tests bench bench_all
#        wab:<k>:<C>:<f32|i16>:<mode>  tools/tune/wide_ab at 2^30 samples, 6 rounds (mode: - self selfhs hs)
#        pt:<file>:<-k expression>     pytest -m gpu on one test file, selected by -k
#        b:<workload>                  one bench.py line (--steps 20 --warmup 5, no CPU baseline)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout-method thread"
run() {  # run <name> <seconds> <command...>
  local name=$1 lim=$2; shift 2
  local t0=$(date +%s)
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "step $name rc=$rc $(( $(date +%s) - t0 )) s"
  if [ $rc -ne 0 ]; then tail -30 "$OUT/$name.log"; exit $rc; fi
}
for s in "$@"; do
  case $s in
    counters) run counters 60 rocprofv3 -L ;;
    fullsize_new) run fullsize_new 400 $PYT --timeout 200 tests/test_gpu_fullsize.py -k "f32_c4_2p30_k2048 or i16_c8_2p30_k2048" ;;
    gloo2) run gloo2 240 $PYT --timeout 200 -m gpu tests/test_bench_launch.py ;;
    ab_i16_mono) run ab_i16_mono 300 tools/tune/wide_ab 30 44100 1 6 0 i16 ;;
    ab_i16_stereo) run ab_i16_stereo 300 tools/tune/wide_ab 30 44100 2 6 0 i16 ;;
    ab_i16_c4) run ab_i16_c4 300 tools/tune/wide_ab 30 44100 4 6 0 i16 ;;
    ab_i16_c8) run ab_i16_c8 300 tools/tune/wide_ab 30 44100 8 6 0 i16 ;;
    gpu_tests) run gpu_tests 1100 $PYT --timeout 300 -m gpu tests/ ;;
    bench) run bench 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench_all) run bench_all 900 python -u bench.py --steps 20 --warmup 5 --all-workloads --no-cpu-baseline ;;
    wab:*) IFS=: read -r _ k c dt mode <<< "$s"
           [ "$mode" = "-" ] && mode=""
           run "wab_${dt}_c${c}_k${k}_${mode:-default}" 300 tools/tune/wide_ab 30 "$k" "$c" 6 0 "$dt" $mode ;;
    pt:*) IFS=: read -r _ f expr <<< "$s"
          run "pt_$(basename "$f" .py)_$(echo "$expr" | tr -c 'A-Za-z0-9' '_' | cut -c1-40)" 1000 \
              $PYT --timeout 300 -m gpu "tests/$f" -k "$expr" ;;
    b:*) w=${s#b:}; run "bench_$w" 200 python -u bench.py --workload "$w" --steps 20 --warmup 5 --no-cpu-baseline ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "session $TAG done"
