#!/bin/bash
# tf_cnn_benchmarks CLI feature sweep on one MI355X at the default precision (fp32) and the 16-bit
# modes: every flag family the reference's runners or users touch, a few steps each. A case passes
# when the run prints "total images/sec". A Python error (rc 1) is recorded and the sweep goes on;
# a time limit, abort or fault (rc 124/134/137/139) ends it, nothing more runs on the GPU.
# SET=2: the second case list (real data, checkpoint timing, comm knobs, 16-bit zoo, inference);
# SET=3: checkpoints across precisions and batch sizes, real data on the other model families.
set -o pipefail
mkdir -p gpurun_out/cli_sweep
OUT=gpurun_out/cli_sweep
SUM=$OUT/summary${SET:-}.txt
: > $SUM
n=0
run() {  # run NAME FLAGS...
  local name=$1; shift
  n=$((n + 1))
  timeout -k 10 240 python -u tf_cnn_benchmarks.py --display_every=2 "$@" > $OUT/$name.log 2>&1
  local rc=$?
  local ips
  ips=$(grep -o "total images/sec: [0-9.]*" $OUT/$name.log | tail -1 | awk '{print $3}')
  if [ $rc -eq 0 ] && [ -n "$ips" ]; then
    echo "PASS $name $ips img/s :: $*" | tee -a $SUM
  else
    echo "FAIL(rc=$rc) $name :: $* :: $(grep -E 'Error|error' $OUT/$name.log | tail -1 | cut -c1-200)" | tee -a $SUM
  fi
  case $rc in 124|134|137|139) echo "stopping: rc $rc" | tee -a $SUM; exit $rc;; esac
  return 0
}
R50="--model=resnet50 --batch_size=64 --num_batches=6 --num_warmup_batches=2"
SMALL="--batch_size=16 --num_batches=4 --num_warmup_batches=1 --autotune=False"
if [ "${SET:-1}" = 3 ]; then  # third set: checkpoints across precisions, real data on the other families
  D=/tmp/hcb_fake_imagenet
  [ -f $D/.done ] || { timeout -k 10 300 python tools/make_fake_imagenet.py $D --shards 4 --per_shard 128 > /dev/null && touch $D/.done; } || exit 1
  rm -rf /tmp/hcb_cli_ckpt3
  run ck_fp32_save $R50 --train_dir=/tmp/hcb_cli_ckpt3 --save_model_steps=3 --optimizer=momentum
  run ck_bf16_resume $R50 --train_dir=/tmp/hcb_cli_ckpt3 --optimizer=momentum --compute_dtype=bf16
  run ck_fp16_resume $R50 --train_dir=/tmp/hcb_cli_ckpt3 --optimizer=momentum --use_fp16=True
  run ck_fp32_fwd $R50 --train_dir=/tmp/hcb_cli_ckpt3 --forward_only=True
  run ck_bs32_resume --model=resnet50 --batch_size=32 --num_batches=4 --num_warmup_batches=1 --train_dir=/tmp/hcb_cli_ckpt3 --optimizer=momentum
  for m in resnet50_v2 googlenet vgg16 alexnet; do
    run ${m}_data_fp32 --model=$m $SMALL --data_dir=$D --data_name=imagenet
    run ${m}_data_fp32_fwd --model=$m $SMALL --data_dir=$D --data_name=imagenet --forward_only=True
  done
  echo "sweep done: $(grep -c ^PASS $SUM) pass, $(grep -c ^FAIL $SUM) fail of $n" | tee -a $SUM
  exit 0
fi
if [ "${SET:-1}" = 2 ]; then  # second set: real data, checkpoint timing, comm knobs, 16-bit zoo, inference
  D=/tmp/hcb_fake_imagenet
  [ -f $D/.done ] || { timeout -k 10 300 python tools/make_fake_imagenet.py $D --shards 4 --per_shard 128 > /dev/null && touch $D/.done; } || exit 1
  rm -rf /tmp/hcb_cli_ckpt2
  run r50_data_fwd $R50 --data_dir=$D --data_name=imagenet --forward_only=True
  run inception3_data --model=inception3 $SMALL --data_dir=$D --data_name=imagenet
  run inception3_data_bf16 --model=inception3 $SMALL --data_dir=$D --data_name=imagenet --compute_dtype=bf16
  run r50_epochs --model=resnet50 --batch_size=64 --num_epochs=0.0003 --num_warmup_batches=2
  run r50_ckpt_secs $R50 --train_dir=/tmp/hcb_cli_ckpt2 --save_model_secs=1
  run r50_repack_spec $R50 --gradient_repacking=4 --all_reduce_spec=nccl --variable_update=horovod
  run r50_summary $R50 --summary_verbosity=1 --benchmark_log_dir=$OUT/bench_logs2 --tf_random_seed=7
  run r50_hvd_cpu $R50 --horovod_device=cpu --variable_update=horovod
  run r50_mkl_kmp $R50 --mkl=True --kmp_blocktime=1 --kmp_affinity=granularity=fine --num_intra_threads=4 --num_inter_threads=2 --xla=True
  run r50v15_fp32 --model=resnet50_v1.5 $SMALL
  run r50v15_fp32_fwd --model=resnet50_v1.5 $SMALL --forward_only=True
  for m in vgg16 googlenet alexnet resnet152_v2 inception3 resnet50_v2; do
    run ${m}_bf16_fwd --model=$m $SMALL --compute_dtype=bf16 --forward_only=True
    run ${m}_fp16 --model=$m $SMALL --use_fp16=True
  done
  echo "sweep done: $(grep -c ^PASS $SUM) pass, $(grep -c ^FAIL $SUM) fail of $n" | tee -a $SUM
  exit 0
fi
rm -rf /tmp/hcb_cli_ckpt
run r50_default $R50
run r50_forward_only $R50 --forward_only=True
run r50_ckpt_save $R50 --train_dir=/tmp/hcb_cli_ckpt --save_model_steps=3 --optimizer=momentum
run r50_ckpt_resume $R50 --train_dir=/tmp/hcb_cli_ckpt --save_model_steps=3 --optimizer=momentum
run r50_trace $R50 --trace_file=$OUT/trace.json
run r50_accuracy_smoothing $R50 --print_training_accuracy=True --label_smoothing=0.1
run r50_eager $R50 --use_hip_graph=False
run r50_sgd_nhwc $R50 --optimizer=sgd --data_format=NHWC
run r50_comm_check $R50 --comm_check=True --variable_update=horovod
run r50_compress_fp16 $R50 --gradient_compression=fp16 --variable_update=horovod
run r50_comm_torch $R50 --comm_engine=torch --variable_update=horovod
run r50_json $R50 --json_summary=$OUT/summary.json --benchmark_log_dir=$OUT/bench_logs
run r50_img160 --model=resnet50 $SMALL --image_size=160
run r50_bf16 $R50 --compute_dtype=bf16
run r50_fp16_autoscale $R50 --use_fp16=True --fp16_enable_auto_loss_scale=True
run r50_fp16_bf16half $R50 --use_fp16=True --half_dtype=bf16
for m in resnet101 resnet152 resnet50_v2 resnet101_v2 resnet152_v2 inception3 trivial vgg11 vgg16 vgg19 alexnet overfeat lenet googlenet; do
  run ${m}_fp32 --model=$m $SMALL
  run ${m}_fp32_fwd --model=$m $SMALL --forward_only=True
done
echo "sweep done: $(grep -c ^PASS $SUM) pass, $(grep -c ^FAIL $SUM) fail of $n" | tee -a $SUM
