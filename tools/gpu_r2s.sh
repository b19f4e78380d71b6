# stem pool kernels (2-D grid argmax backward, unrolled 3x3 BN+ReLU+max-pool): tests, bench, kernel trace
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_zoo_gpu.py tests/test_stem_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s_pytest.log 2>&1 || { tail -30 gpurun_out/s_pytest.log; exit 1; }
tail -1 gpurun_out/s_pytest.log
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/s_bench.json 2> gpurun_out/s_bench.err || { tail -20 gpurun_out/s_bench.err; exit 1; }
  echo "bench $(python -c 'import json;d=json.load(open("gpurun_out/s_bench.json"));print(d["value"], d["ms_per_step"])')"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/s_prof" -o run -- python "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/s_prof.log" 2>&1 || { echo "rocprof failed"; tail -5 "$GRAFT_REPO_ROOT/gpurun_out/s_prof.log"; exit 1; }
echo prof done
