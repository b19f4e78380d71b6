#!/bin/bash
# Iteration loop on the GPU box: build, GPU tests, per-layer conv bench (tuned), bench, rocprof.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -q -s --maxfail=10 -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
  [ $rc -le 1 ] || exit $rc
fi
if [ "${CONV_BENCH:-1}" = "1" ]; then
  timeout -k 10 600 python tools/conv_bench.py --model resnet50 --batch 64 --tune --json gpurun_out/conv_bench.json > gpurun_out/conv_bench.log 2>&1 || { echo conv_bench failed; tail -20 gpurun_out/conv_bench.log; exit 1; }
  tail -1 gpurun_out/conv_bench.log
fi
if [ -n "${AB_ENV:-}" ]; then  # A/B: the same bench with an env toggle (e.g. AB_ENV=HCB_FUSE_BN_BWD=0)
  env $AB_ENV timeout -k 10 400 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_ab.log 2>&1 || { echo "bench A/B failed"; tail -40 gpurun_out/bench_ab.log; exit 1; }
  echo "A/B ($AB_ENV):"; tail -1 gpurun_out/bench_ab.log
fi
timeout -k 10 400 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
cp azure_hc_intel_tf_amd/tuned/mi355x.json gpurun_out/tuned_mi355x.json 2>/dev/null
if [ "${PROF:-1}" = "1" ]; then
  cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof.log; exit 1; }
  echo "prof done"
fi
