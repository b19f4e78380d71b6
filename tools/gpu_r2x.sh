# 128x64 / 64x128 register-staged weight-grad tiles: tests, wgrad retune, per-layer A/B, bench
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad" -x -q --timeout 120 --timeout-method thread > gpurun_out/x_test.log 2>&1 || { tail -30 gpurun_out/x_test.log; exit 1; }
tail -1 gpurun_out/x_test.log
timeout -k 10 900 python -u tools/retune_wgrad.py > gpurun_out/x_retune.log 2>&1 || { tail -20 gpurun_out/x_retune.log; exit 1; }
grep "tuned [0-9]* problems" gpurun_out/x_retune.log
timeout -k 10 300 python -u tools/wgrad_ab.py > gpurun_out/x_wgrad_ab.txt 2>&1 || { tail -20 gpurun_out/x_wgrad_ab.txt; exit 1; }
cat gpurun_out/x_wgrad_ab.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/x_bench.json 2> gpurun_out/x_bench.err || { tail -20 gpurun_out/x_bench.err; exit 1; }
  echo "bench $(python -c 'import json;d=json.load(open("gpurun_out/x_bench.json"));print(d["value"], d["ms_per_step"])')"
done
