set -o pipefail
mkdir -p gpurun_out
for L in stage1/block1/shortcut stage1/block1/conv2 stage1/block2/conv1 stage2/block1/conv3; do
 for F in --fp32 ""; do
  for R in -1 0 8 64; do
   timeout -k 10 120 python tools/layer_probe.py $F --layer $L --op fwd --reps 40 --stats_r $R 2>&1 | grep -v amdgpu.ids | sed "s/^/R=$R $F /" || exit 1
  done
 done
done
