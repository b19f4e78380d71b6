# persistent short-K plane GEMM (cfg 18-22) against its twin cfg, isolated per layer (tools/layer_probe.py)
set -o pipefail
for spec in "stage1/block1/shortcut:fwd:15:18" "stage1/block1/conv3:fwd:15:18" "stage1/block2/conv1:fwd:14:19" \
            "stage1/block1/conv1:fwd:16:20" "stage1/block1/conv1:fwd:17:21" "stage2/block1/conv3:fwd:14:19" \
            "stage2/block1/conv1:fwd:16:20" "stage2/block2/conv1:fwd:14:19" "stage3/block1/conv3:fwd:7:22" \
            "stage1/block1/conv3:dgrad:14:19" "stage1/block1/conv2:fwd:14:19"; do
  IFS=: read L OP A B <<< "$spec"
  for c in $A $B $A $B; do
    timeout -k 10 120 python tools/layer_probe.py --fp32 --layer $L --op $OP --reps 40 --cfg $c 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
