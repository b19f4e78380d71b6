#!/bin/bash
# the stage-3 1x1 short-K problem (M 12544, N 1024, K 256: conv3 forward / conv1 data gradient) on every
# tile family, isolated (tools/layer_probe.py --fp32)
set -o pipefail
mkdir -p gpurun_out/r6v
for c in 17 21 16 20 15 18 14 19 7 22 8 13 27; do
  timeout -k 10 60 python tools/layer_probe.py --fp32 --layer stage3/block2/conv3 --op fwd --cfg $c --reps 40 2>&1 \
    | grep -v amdgpu.ids >> gpurun_out/r6v/sk.txt || exit 1
done
for c in 17 21 18 22 8; do
  timeout -k 10 60 python tools/layer_probe.py --fp32 --layer stage3/block2/conv1 --op dgrad --cfg $c --reps 40 2>&1 \
    | grep -v amdgpu.ids >> gpurun_out/r6v/sk.txt || exit 1
done
cat gpurun_out/r6v/sk.txt
