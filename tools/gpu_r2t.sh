# weight-grad two-set register prefetch: tests, per-layer A/B, bench
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_test.log 2>&1 || { tail -30 gpurun_out/t_test.log; exit 1; }
tail -1 gpurun_out/t_test.log
timeout -k 10 300 python -u tools/wgrad_ab.py > gpurun_out/t_wgrad_ab.txt 2>&1 || { tail -20 gpurun_out/t_wgrad_ab.txt; exit 1; }
cat gpurun_out/t_wgrad_ab.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/t_bench.json 2> gpurun_out/t_bench.err || { tail -20 gpurun_out/t_bench.err; exit 1; }
  echo "bench $(python -c 'import json;d=json.load(open("gpurun_out/t_bench.json"));print(d["value"], d["ms_per_step"])')"
done
