# stream-K plane GEMM (cfg 23-30) against the tuned plan, isolated per layer (tools/layer_probe.py),
# interleaved twice. Output lines: layer op cfg us TF.
set -o pipefail
for spec in "stage3/block1/conv2:fwd:8:29:30:28" "stage4/block2/conv2:fwd:8,2:29:30" "stage2/block2/conv2:fwd:8:29:30" \
            "stage3/block1/shortcut:fwd:11:29:30" "stage3/block2/conv3:fwd:22:29:30" "stage1/block2/conv2:fwd:19:29" \
            "stage4/block1/shortcut:fwd:11,1:29:30" "stage4/block2/conv3:fwd:22:29:30"; do
  IFS=: read L OP A B C D <<< "$spec"
  for r in 1 2; do
    for c in $A $B $C $D; do
      timeout -k 10 120 python tools/layer_probe.py --fp32 --layer $L --op $OP --reps 40 --cfg $c 2>&1 | grep -v amdgpu.ids || exit 1
    done
  done
done
