#!/bin/bash
# Secondary GPU checks: tests, tools, other models' throughput (run via gpurun).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
  [ $rc -le 1 ] || exit $rc
fi
timeout -k 10 120 python tools/env_report.py --json gpurun_out/env_report.json > gpurun_out/env_report.txt 2>&1 || { echo env_report failed; tail gpurun_out/env_report.txt; exit 1; }
head -12 gpurun_out/env_report.txt
timeout -k 10 300 tools/rccl_bench/rccl_allreduce_bench -n 1 -b 1K -e 256M -f 4 -d float -j gpurun_out/rccl_bench_n1.json > gpurun_out/rccl_bench_n1.txt 2>&1 || { echo rccl bench failed; tail gpurun_out/rccl_bench_n1.txt; exit 1; }
tail -3 gpurun_out/rccl_bench_n1.txt
for spec in ${MODELS:-resnet152:128 inception3:64 resnet101:64 resnet50_v1.5:64}; do
  IFS=: read m b <<< "$spec"
  timeout -k 10 600 python bench.py --model $m --batch_size $b --steps 20 --warmup 5 > gpurun_out/bench_$m.log 2>&1 || { echo "bench $m failed"; tail -20 gpurun_out/bench_$m.log; exit 1; }
  tail -1 gpurun_out/bench_$m.log | cut -c1-200
done
cp azure_hc_intel_tf_amd/tuned/mi355x.json gpurun_out/tuned_mi355x.json 2>/dev/null
echo "gpu_misc done"
