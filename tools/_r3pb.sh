set -o pipefail
mkdir -p gpurun_out
TAG=r3pb bash tools/gpu_run.sh tests:tests/test_conv3x3_patch_gpu.py || exit 1
timeout -k 10 300 python -u tools/patch_sweep.py --stages 1 --cfgs 1,2,5,6,10,19,20 > gpurun_out/r3pb_sweep.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/patch_sweep.py --stages 1 --cfgs 1,2,5,6,10,19,20 --pass dgrad >> gpurun_out/r3pb_sweep.txt 2>&1 || exit 1
