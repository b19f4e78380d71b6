set -o pipefail
mkdir -p gpurun_out
export HCB_TUNE_REPS=20
timeout -k 10 900 python -u tools/retune_conv.py resnet152 inception3 resnet101 resnet50_v1.5 > gpurun_out/r3k_tune_conv.log 2>&1 || exit 1
timeout -k 10 900 python -u tools/retune_wgrad.py > gpurun_out/r3k_tune_wgrad.log 2>&1 || exit 1
cp azure_hc_intel_tf_amd/tuned/mi355x.json gpurun_out/r3k_cache.json
TAG=r3k bash tools/gpu_run.sh bench prof
