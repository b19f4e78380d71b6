set -o pipefail
mkdir -p gpurun_out
python __graft_entry__.py > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 900 python -m pytest tests -q -s --maxfail=10 -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 600 python tools/conv_bench.py --model resnet50 --batch 64 --json gpurun_out/conv_bench.json > gpurun_out/conv_bench.log 2>&1 || { echo conv_bench failed; tail -20 gpurun_out/conv_bench.log; exit 1; }
tail -3 gpurun_out/conv_bench.log
timeout -k 10 400 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench.log; exit 1; }
tail -2 gpurun_out/bench.log
cp azure_hc_intel_tf_amd/tuned/mi355x.json gpurun_out/tuned_mi355x.json 2>/dev/null
