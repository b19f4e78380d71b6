#!/bin/bash
# The 1-GPU points of BASELINE.json's configs (run via gpurun; the multi-GPU points come from the
# driver's 8-GPU scaling run):
#   2: ResNet-50 bs=256 bf16, 1x MI355X                      (bench.py)
#   3: ResNet-50 bs=64/worker, 1 worker                      (bench.py, the headline)
#   4: Inception-v3 bs=64/worker, 1 worker                   (bench.py)
#   5: ResNet-152 fp16 bs=128/worker, loss scaling, fp16 gradient compression, 1 worker
#      (tf_cnn_benchmarks.py CLI with the reference's flags)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/cfg_$name.log 2>&1 || { echo "$name failed"; tail -20 gpurun_out/cfg_$name.log; exit 1; }
  echo "== $name"; grep -E '^\{|total images/sec' gpurun_out/cfg_$name.log | tail -1 | cut -c1-400
}
run c2_resnet50_bs256 600 python bench.py --batch_size 256 --steps 20 --warmup 5
run c3_resnet50_bs64 400 python bench.py --steps 50 --warmup 10
run c4_inception3_bs64 600 python bench.py --model inception3 --batch_size 64 --steps 20 --warmup 5
run c5_resnet152_fp16_bs128 900 python tf_cnn_benchmarks.py --model=resnet152 --batch_size=128 --num_batches=30 \
    --num_warmup_batches=10 --display_every=10 --optimizer=momentum --variable_update=horovod --use_fp16 \
    --fp16_enable_auto_loss_scale --gradient_compression=fp16 --device=gpu
cp azure_hc_intel_tf_amd/tuned/mi355x.json gpurun_out/tuned_mi355x.json
echo "baseline configs done"
