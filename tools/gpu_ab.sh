#!/bin/bash
# A/B on the GPU box: targeted tests, then bench.py with and without an env toggle, then a
# rocprofv3 kernel summary of the default configuration.
#   AB_ENV="HCB_WGRAD_STREAM=0" TESTS="tests/test_kernels_gpu.py -k pack" bash tools/gpu_ab.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread $TESTS > gpurun_out/pytest_ab.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pytest_ab.log; exit 1; }
  tail -2 gpurun_out/pytest_ab.log
fi
STEPS=${STEPS:-30}
BENCH_ARGS=${BENCH_ARGS:-}
timeout -k 10 400 python bench.py --steps $STEPS --warmup 5 $BENCH_ARGS > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench.log; exit 1; }
echo "default:"; tail -1 gpurun_out/bench.log
cp azure_hc_intel_tf_amd/tuned/mi355x.json gpurun_out/tuned_mi355x.json  # autotune results of this box
if [ -n "${AB_ENV:-}" ]; then
  env $AB_ENV timeout -k 10 400 python bench.py --steps $STEPS --warmup 5 $BENCH_ARGS > gpurun_out/bench_ab.log 2>&1 || { echo "bench A/B failed"; tail -40 gpurun_out/bench_ab.log; exit 1; }
  echo "A/B ($AB_ENV):"; tail -1 gpurun_out/bench_ab.log
fi
if [ "${PROF:-1}" = "1" ]; then
  cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 $BENCH_ARGS > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof.log; exit 1; }
  echo "prof done"
fi
cp azure_hc_intel_tf_amd/tuned/mi355x.json gpurun_out/tuned_mi355x.json 2>/dev/null || true
