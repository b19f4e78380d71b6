set -o pipefail
mkdir -p gpurun_out
TAG=r3fd bash tools/gpu_run.sh tests:tests/test_conv3x3_patch_gpu.py,tests/test_kernels_gpu.py || exit 1
timeout -k 10 300 python -u tools/patch_sweep.py --cfgs 1,2,5,6,7,13,14,16,17,18,19,20,21 --top 6 > gpurun_out/r3fd_sweep.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/patch_sweep.py --cfgs 1,2,5,6,7,13,14,16,17,18,19,20,21 --top 6 --pass dgrad >> gpurun_out/r3fd_sweep.txt 2>&1 || exit 1
