set -o pipefail
mkdir -p gpurun_out/r6t
for spec in "stage3/block1/conv2 8,1 10,1 10,2 11,1 11,2 9,1 9,2 7,1" "stage2/block2/conv2 8,1 10,1 10,2 11,1 9,1" "stage4/block2/conv2 8,2 10,2 10,4 11,2 11,4 9,2"; do
  set -- $spec; L=$1; shift
  for c in "$@"; do
    timeout -k 10 60 python tools/layer_probe.py --fp32 --layer $L --op fwd --cfg $c --reps 40 2>&1 | grep -v amdgpu.ids >> gpurun_out/r6t/cfg.txt || exit 1
  done
done
cat gpurun_out/r6t/cfg.txt
