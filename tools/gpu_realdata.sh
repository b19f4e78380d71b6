#!/bin/bash
# Real-data (--data_dir) path on the GPU box: write an ImageNet-format TFRecord set of random
# JPEGs, then train ResNet-50 from it through the native prefetch -> Pillow decode -> GPU
# preprocess pipeline with the tf_cnn_benchmarks CLI. EXTRA= appends flags (e.g. --compute_dtype=bf16),
# TAG= suffixes the log name.
set -o pipefail
mkdir -p gpurun_out
D=/tmp/hcb_fake_imagenet
[ -f $D/.done ] || { timeout -k 10 300 python tools/make_fake_imagenet.py $D --shards 8 --per_shard 256 > /dev/null && touch $D/.done; } || exit 1
timeout -k 10 600 python tf_cnn_benchmarks.py --model=resnet50 --batch_size=64 --num_batches=40 --num_warmup_batches=5 \
   --display_every=10 --optimizer=momentum --variable_update=horovod --data_dir=$D --data_name=imagenet \
   --num_decode_threads=${DECODE:-16} --datasets_num_private_threads=4 ${EXTRA:-} > gpurun_out/realdata${TAG:-}.log 2>&1 || { tail -30 gpurun_out/realdata${TAG:-}.log; exit 1; }
grep -E "Dataset|images/sec|Reading" gpurun_out/realdata${TAG:-}.log
