# fused BN-backward epilogue prefetch chunk (HCB_BNB_CH 4 default / 2 / 1) A/B, alternating bench runs
mkdir -p gpurun_out
export TMPDIR=/tmp
HCB_KERNELS_SO=abvar/ch1/_hcb_kernels.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "fused_bn_backward" -x -q --timeout 120 --timeout-method thread > gpurun_out/ac_t1.log 2>&1 || { tail -20 gpurun_out/ac_t1.log; exit 1; }
tail -1 gpurun_out/ac_t1.log
for r in 1 2; do for v in def ch2 ch1; do
  if [ $v = def ]; then so=""; else so=abvar/$v/_hcb_kernels.so; fi
  HCB_KERNELS_SO=$so timeout -k 10 300 python bench.py > gpurun_out/ac_b.json 2> gpurun_out/ac_b.err || { tail -20 gpurun_out/ac_b.err; exit 1; }
  echo "$v $(python -c 'import json;d=json.load(open("gpurun_out/ac_b.json"));print(d["value"], d["ms_per_step"])')"
done; done
