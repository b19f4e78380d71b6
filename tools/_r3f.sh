set -o pipefail
mkdir -p gpurun_out
for v in main b128 a1 a2 a3; do
  if [ $v = main ]; then so=""; else so=abv/$v/_hcb_kernels.so; fi
  echo "== variant $v" >> gpurun_out/r3f_ab.txt
  HCB_KERNELS_SO=$so timeout -k 10 300 python -u tools/patch_sweep.py --cfgs 7,13,14,16,17,18,19,20,21 --top 20 >> gpurun_out/r3f_ab.txt 2>&1 || exit 1
done
