set -o pipefail
L="python -u tools/layer_probe.py --fp32 --layer stage3/block1/conv2 --op fwd --reps 50"
for c in 8,1 8,-256 8,-512 7,1 7,-256 11,-256 10,-256 14,-512 14,1 17,-768 17,1; do
  timeout -k 10 60 $L --cfg $c 2>&1 | grep -v amdgpu || exit 1
done
L="python -u tools/layer_probe.py --fp32 --layer stage2/block1/conv2 --op fwd --reps 50"
for c in 10,1 10,-256 10,-512 7,-256 17,-768 17,1; do
  timeout -k 10 60 $L --cfg $c 2>&1 | grep -v amdgpu || exit 1
done
