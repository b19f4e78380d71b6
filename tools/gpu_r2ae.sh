# fused BN-backward parameters staged in LDS at kernel start (variant build abvar2/bnbp): tests, probe, bench A/B
mkdir -p gpurun_out
export TMPDIR=/tmp
V=abvar2/bnbp/_hcb_kernels.so
HCB_KERNELS_SO=$V timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_dgrad_phases_gpu.py tests/test_fused_resbn_gpu.py tests/test_model_gpu.py tests/test_determinism_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ae_pytest.log 2>&1 || { tail -30 gpurun_out/ae_pytest.log; exit 1; }
tail -1 gpurun_out/ae_pytest.log
HCB_KERNELS_SO=$V timeout -k 10 300 python -u tools/bnb_probe.py > gpurun_out/ae_bnb_probe.txt 2>&1 || { tail -20 gpurun_out/ae_bnb_probe.txt; exit 1; }
grep -E "==|cfg  [015]:|cfg 10" gpurun_out/ae_bnb_probe.txt
for r in 1 2; do for v in def var; do
  if [ $v = def ]; then so=""; else so=$V; fi
  HCB_KERNELS_SO=$so timeout -k 10 300 python bench.py > gpurun_out/ae_b.json 2> gpurun_out/ae_b.err || { tail -20 gpurun_out/ae_b.err; exit 1; }
  echo "$v $(python -c 'import json;d=json.load(open("gpurun_out/ae_b.json"));print(d["value"], d["ms_per_step"])')"
done; done
