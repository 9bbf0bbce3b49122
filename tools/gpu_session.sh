#!/bin/bash
# One GPU session on the gpurun box.  Every GPU step has its own time limit;
# a crash / abort / timeout (exit >= 124 or signal) ends the session there.
# Usage: tools/gpu_session.sh <tag> [steps...]   steps: test bench prof pmc smoke
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { # exit codes that mean the GPU step did not end normally
  local rc=$1
  [ "$rc" -ge 124 ] && return 0
  return 1
}
run() { # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/session.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/session.log"
  tail -5 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL rc=$rc in $name; stopping" | tee -a "$OUT/session.log"; exit $rc; fi
  return 0
}
for step in "$@"; do
  case $step in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    test) run pytest_gpu 900 python -m pytest tests -m gpu -q --maxfail=30 -p no:cacheprovider ;;
    testx) run pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread \
            -p no:cacheprovider ;;
    testm) run pytest_gpu 1000 python -u -m pytest tests -m gpu -v --maxfail=10 --timeout 200 --timeout-method thread \
            -p no:cacheprovider ;;
    bench) run bench 400 python bench.py --steps 20 --warmup 5 --all-workloads ;;
    prof) run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
            python bench.py --steps 10 --warmup 3 --no-cpu-baseline --all-workloads ;;
    pmc) run pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
            python bench.py --steps 5 --warmup 2 --no-cpu-baseline --all-workloads &&
         run pmc_write 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
            python bench.py --steps 5 --warmup 2 --no-cpu-baseline --all-workloads ;;
    check) run check1 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --check --all-workloads ;;
    dist) run dist2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
            --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --check &&
          run dist4 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
            --master-port 29512 bench.py --gpus 4 --steps 3 --warmup 1 --dist-backend gloo --check ;;
    dist2) run pytest_dist2 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -k rounding -s -q \
            --timeout 170 --timeout-method thread -p no:cacheprovider ;;
    full) run pytest_full 900 python -u -m pytest tests/test_gpu_fullsize.py tests/test_bench_launch.py -m gpu -x -v \
            --timeout 170 --timeout-method thread -p no:cacheprovider ;;
    # the driver's exact bench command, then the same command under the kernel tracer
    drv) run drv_bench 400 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    drvprof) run drv_prof 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/drvprof" -o run -- \
            python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    *) echo "unknown step $step" ;;
  esac
done
echo "session done" | tee -a "$OUT/session.log"
