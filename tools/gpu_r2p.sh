# row-incremental weight-grad loaders: tests, per-layer A/B, wgrad retune, bench A/B
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad" -x -q --timeout 120 --timeout-method thread > gpurun_out/p_test.log 2>&1 || { tail -30 gpurun_out/p_test.log; exit 1; }
tail -1 gpurun_out/p_test.log
timeout -k 10 300 python -u tools/wgrad_ab.py > gpurun_out/p_wgrad_ab.txt 2>&1 || { tail -20 gpurun_out/p_wgrad_ab.txt; exit 1; }
cat gpurun_out/p_wgrad_ab.txt
timeout -k 10 900 python -u tools/retune_wgrad.py > gpurun_out/p_retune.log 2>&1 || { tail -20 gpurun_out/p_retune.log; exit 1; }
grep "tuned [0-9]* problems" gpurun_out/p_retune.log
timeout -k 10 300 python -u tools/wgrad_ab.py > gpurun_out/p_wgrad_ab_tuned.txt 2>&1 || { tail -20 gpurun_out/p_wgrad_ab_tuned.txt; exit 1; }
tail -1 gpurun_out/p_wgrad_ab_tuned.txt
for ri in 1 0 2 1 0; do
  HCB_WGRAD_RI=$ri timeout -k 10 300 python bench.py > gpurun_out/p_bench.json 2> gpurun_out/p_bench.err || { tail -20 gpurun_out/p_bench.err; exit 1; }
  echo "HCB_WGRAD_RI=$ri $(python -c 'import json;d=json.load(open("gpurun_out/p_bench.json"));print(d["value"], d["ms_per_step"])')"
done
