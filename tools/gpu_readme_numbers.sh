#!/bin/bash
# Every 1-GPU throughput the README quotes, in one run (gpurun): BASELINE configs 2-5, the
# PyTorch+MIOpen comparison point, the model zoo. Output: gpurun_out/readme_numbers.log (ZOO_ONLY=1: readme_numbers_zoo.log)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/readme_numbers${ZOO_ONLY:+_zoo}.log
: > $OUT
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/rn_$name.log 2>&1 || { echo "$name failed" | tee -a $OUT; tail -20 gpurun_out/rn_$name.log; exit 1; }
  echo "== $name: $*" >> $OUT
  grep -E '^\{|total images/sec|images/sec:' gpurun_out/rn_$name.log | tail -1 | cut -c1-600 >> $OUT
  tail -1 $OUT | cut -c1-200
}
if [ -z "$ZOO_ONLY" ]; then  # ZOO_ONLY=1: only the zoo rows (MODELS=" " / FP32_MODELS=" ": none of them)
run c3_resnet50_bs64 300 python bench.py --steps 60 --warmup 10   # fp32 headline + bf16 secondary
run c2_resnet50_bs256 400 python bench.py --batch_size 256 --compute_dtype bf16 --secondary none --steps 20 --warmup 5
run c2_resnet50_bs256_fp32 400 python bench.py --batch_size 256 --compute_dtype fp32 --secondary none --steps 10 --warmup 3
run c4_inception3_bs64 400 python bench.py --model inception3 --batch_size 64 --compute_dtype bf16 --secondary none \
    --steps 20 --warmup 5
run c4_inception3_bs64_fp32 400 python bench.py --model inception3 --batch_size 64 --compute_dtype fp32 --secondary none \
    --steps 20 --warmup 5
run c5_resnet152_fp16_bs128 600 python tf_cnn_benchmarks.py --model=resnet152 --batch_size=128 --num_batches=30 \
    --num_warmup_batches=10 --display_every=10 --optimizer=momentum --variable_update=horovod --use_fp16 \
    --fp16_enable_auto_loss_scale --device=gpu
run miopen_eager_resnet50_bs64 400 python tools/torch_resnet_baseline.py --batch 64 --steps 30
fi
for spec in ${MODELS:-resnet101:64 resnet50_v1.5:64 resnet50_v2:64 vgg16:64 googlenet:128 alexnet:512 overfeat:128}; do
  IFS=: read m b <<< "$spec"
  run zoo_$m 400 python bench.py --model $m --batch_size $b --compute_dtype bf16 --secondary none --steps 20 --warmup 5
done
for spec in ${FP32_MODELS:-resnet50_v2:64 resnet101:64 vgg16:64 googlenet:128 alexnet:512}; do  # the zoo at fp32 on the HIP kernels
  IFS=: read m b <<< "$spec"
  run zoo32_$m 400 python bench.py --model $m --batch_size $b --compute_dtype fp32 --secondary none --steps 20 --warmup 5
done
echo "readme numbers done" >> $OUT
