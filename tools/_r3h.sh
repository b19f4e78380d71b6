set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3h_ab.txt
cp azure_hc_intel_tf_amd/tuned/mi355x.json /tmp/cache0.json
for v in main fs2; do
  if [ $v = main ]; then so=""; else so=abv/$v/_hcb_kernels.so; fi
  cp /tmp/cache0.json azure_hc_intel_tf_amd/tuned/mi355x.json
  HCB_KERNELS_SO=$so timeout -k 10 600 python -u tools/retune_conv.py resnet50 > gpurun_out/r3h_tune_$v.log 2>&1 || exit 1
  cp azure_hc_intel_tf_amd/tuned/mi355x.json gpurun_out/r3h_cache_$v.json
  for r in 1 2; do
    echo "bench $v: $(HCB_KERNELS_SO=$so timeout -k 10 300 python bench.py --steps 40 --warmup 10 | cut -c1-150)" >> $O || exit 1
  done
done
