#!/bin/bash
# One gpurun call (no build on the box: the in-tree .so files travel with the snapshot).
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
STEP=${1:-all}
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -25 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || { echo "$name failed rc=$rc"; exit $rc; }
}
case "$STEP" in
  all|tests)
    run smoke 300 python __graft_entry__.py smoke
    run pytest_gpu 1100 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ;;
esac
case "$STEP" in
  all|bench)
    run bench1 400 python bench.py --steps 30 --warmup 5
    run bench_dp1 400 python bench.py --steps 30 --warmup 5 --force_dp_path
    HCB_BENCH_ONE_DEVICE=1 HCB_BENCH_BACKEND=gloo run bench_gloo2 500 python bench.py --gpus 2 --steps 5 --warmup 3 --no_tune
    run bench_gpus8_refused 120 bash -c '! python bench.py --gpus 8 --steps 1 --warmup 0' ;;
esac
case "$STEP" in
  all|prof)
    cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { echo "rocprof failed"; tail -30 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 1; }
    echo "prof done" ;;
esac
