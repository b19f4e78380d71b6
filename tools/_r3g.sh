set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3g_ab.txt
for v in main fs; do
  if [ $v = main ]; then so=""; else so=abv/$v/_hcb_kernels.so; fi
  echo "== variant $v" >> $O
  HCB_KERNELS_SO=$so timeout -k 10 300 python -u tools/patch_sweep.py --cfgs 2,5,6,7,13,14,16,17,18,19,20,21 --top 8 >> $O 2>&1 || exit 1
done
for r in 1 2; do for v in main fs; do
  if [ $v = main ]; then so=""; else so=abv/$v/_hcb_kernels.so; fi
  echo "bench $v: $(HCB_KERNELS_SO=$so timeout -k 10 300 python bench.py --steps 40 --warmup 10 | cut -c1-150)" >> $O || exit 1
done; done
