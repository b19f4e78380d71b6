# KU=2 LDS-DMA configs (22-26): kernel tests, 3x3 sweep, retune, bench, kernel profile
set -o pipefail
mkdir -p gpurun_out
TAG=r3w bash tools/gpu_run.sh tests:tests/test_kernels_gpu.py,tests/test_conv3x3_patch_gpu.py || exit 1
timeout -k 10 300 python -u tools/patch_sweep.py --cfgs 2,5,6,7,13,14,16,18,22,23,24,25,26 --top 8 > gpurun_out/r3w_sweep.txt 2>&1 || exit 1
export HCB_TUNE_REPS=20
timeout -k 10 900 python -u tools/retune_conv.py resnet50 resnet152 inception3 resnet101 resnet50_v1.5 > gpurun_out/r3w_tune.log 2>&1 || exit 1
cp azure_hc_intel_tf_amd/tuned/mi355x.json gpurun_out/r3w_cache.json
TAG=r3w bash tools/gpu_run.sh bench prof
