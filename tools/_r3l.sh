# round-3 verification run: smoke, whole GPU suite, bench, per-layer conv table vs MIOpen, PMC of the
# stage-2/3 3x3 convs at their tuned configs
set -o pipefail
mkdir -p gpurun_out
PYTEST_X= TAG=r3l bash tools/gpu_run.sh smoke tests bench || exit 1
timeout -k 10 600 python -u tools/conv_bench.py --model resnet50 --batch 64 > gpurun_out/r3l_conv_bench.txt 2>&1 || exit 1
LAYERS="stage2/block1/conv2:fwd:- stage3/block1/conv2:fwd:- stage2/block1/conv2:dgrad:- stage3/block1/conv2:dgrad:-" timeout 900 bash tools/prof_conv.sh && python tools/pmc_summary.py gpurun_out/pmc > gpurun_out/r3l_pmc.txt
