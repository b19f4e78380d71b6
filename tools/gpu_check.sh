#!/bin/bash
# One gpurun call: build, smoke, GPU tests, bench, rocprof kernel stats. Each GPU step has its
# own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
STEP=${1:-all}
python __graft_entry__.py > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -30 gpurun_out/build.log; exit 1; }
if [ "$STEP" = "all" ] || [ "$STEP" = "tests" ]; then
  timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -40 gpurun_out/smoke.log; exit 1; }
  timeout -k 10 1200 python -m pytest tests -q -s --maxfail=10 -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -30 gpurun_out/pytest_gpu.log
  grep -E "median grad" gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || [ "$STEP" = "all" ] || exit $rc
fi
if [ "$STEP" = "all" ] || [ "$STEP" = "bench" ]; then
  timeout -k 10 400 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench.log; exit 1; }
  cat gpurun_out/bench.log
  timeout -k 10 300 python tools/torch_resnet_baseline.py > gpurun_out/torch_baseline.log 2>&1; tail -3 gpurun_out/torch_baseline.log
  cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof.log; exit 1; }
  echo "prof done"
fi
