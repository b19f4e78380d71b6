# A/B: weight-grad kernel with every transposed LDS read of a k-step issued before its MFMAs (abv/ws)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3ws_ab.txt
: > $O
for v in main ws; do
  if [ $v = main ]; then so=""; else so=abv/$v/_hcb_kernels.so; fi
  HCB_KERNELS_SO=$so timeout -k 10 600 python -u tools/conv_bench.py --model resnet50 --batch 64 --no_miopen > gpurun_out/r3ws_cb_$v.txt 2>&1 || exit 1
  echo "$v conv_bench: $(tail -1 gpurun_out/r3ws_cb_$v.txt)" >> $O
done
for r in 1 2 3; do for v in main ws; do
  if [ $v = main ]; then so=""; else so=abv/$v/_hcb_kernels.so; fi
  HCB_KERNELS_SO=$so timeout -k 10 300 python bench.py --steps 40 --warmup 10 > /tmp/b.json || exit 1
  echo "bench $v: $(python -c "import json;d=json.load(open('/tmp/b.json'));print(d['value'], d['ms_per_step'])")" >> $O
done; done
