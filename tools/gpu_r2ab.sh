# register-staged conv kernel: one LDS buffer pair for single-k-step GEMMs: tests, bench, fwd/dgrad retune (all configs), bench
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_zoo_gpu.py tests/test_fp16_native_gpu.py tests/test_dgrad_phases_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
tail -1 gpurun_out/ab_pytest.log
timeout -k 10 300 python bench.py > gpurun_out/ab_bench.json 2> gpurun_out/ab_bench.err || { tail -20 gpurun_out/ab_bench.err; exit 1; }
echo "bench (old tuning) $(python -c 'import json;d=json.load(open("gpurun_out/ab_bench.json"));print(d["value"], d["ms_per_step"])')"
timeout -k 10 900 python -u tools/retune_conv.py resnet50 resnet152 inception3 resnet101 resnet50_v1.5 > gpurun_out/ab_retune.log 2>&1 || { tail -20 gpurun_out/ab_retune.log; exit 1; }
grep "tuned [0-9]* problems\|dropped" gpurun_out/ab_retune.log
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/ab_bench.json 2> gpurun_out/ab_bench.err || { tail -20 gpurun_out/ab_bench.err; exit 1; }
  echo "bench (retuned) $(python -c 'import json;d=json.load(open("gpurun_out/ab_bench.json"));print(d["value"], d["ms_per_step"])')"
done
