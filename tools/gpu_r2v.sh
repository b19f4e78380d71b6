# BN apply: shifts / affine params prefetched before the replica reduction: tests, BN probe, bench
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_bn_shift_gpu.py tests/test_fused_resbn_gpu.py tests/test_stem_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v_pytest.log 2>&1 || { tail -30 gpurun_out/v_pytest.log; exit 1; }
tail -1 gpurun_out/v_pytest.log
timeout -k 10 300 python -u tools/bn_probe.py > gpurun_out/v_bn_probe.txt 2>&1 || { tail -20 gpurun_out/v_bn_probe.txt; exit 1; }
grep -v amdgpu gpurun_out/v_bn_probe.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/v_bench.json 2> gpurun_out/v_bench.err || { tail -20 gpurun_out/v_bench.err; exit 1; }
  echo "bench $(python -c 'import json;d=json.load(open("gpurun_out/v_bench.json"));print(d["value"], d["ms_per_step"])')"
done
