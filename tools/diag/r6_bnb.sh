#!/bin/bash
# persistent BNB epilogue: tests, isolated probes (persistent vs twin), then the A/A band
set -o pipefail
O=gpurun_out/r6l
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fp32_native_gpu.py \
  -k "persistent_fused or fused_bn_backward" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
for spec in "stage1/block1/conv3 16 20" "stage1/block1/conv3 14 19" "stage1/block1/conv2 14 19" "stage1/block2/conv1 16 20" "stage2/block1/conv3 13 18"; do
  set -- $spec
  for c in $2 $3; do
    for b in 1 2; do
      timeout -k 10 60 python tools/layer_probe.py --fp32 --op dgrad --layer $1 --cfg $c --bnb $b --reps 100 >> $O/probe.txt 2>&1 || exit 1
    done
  done
  timeout -k 10 60 python tools/layer_probe.py --fp32 --op dgrad --layer $1 --cfg $3 --reps 100 >> $O/probe.txt 2>&1 || exit 1
done
cat $O/probe.txt
