# multi-GPU path rehearsal on one GPU: the forced data-parallel step on a 1-rank RCCL communicator, and a
# 2-rank gloo run sharing the GPU (bench.py's own spawn path)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3dp.txt
: > $O
timeout -k 10 300 python bench.py --force_dp_path --steps 30 --warmup 10 > /tmp/a.json 2> gpurun_out/r3dp_a.err || exit 1
echo "force_dp_path (1-rank RCCL, segmented overlap graph): $(cut -c1-700 /tmp/a.json)" >> $O
HCB_BENCH_ONE_DEVICE=1 HCB_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 3 > /tmp/b.json 2> gpurun_out/r3dp_b.err || exit 1
echo "gloo x2 on one GPU (spawned ranks): $(cut -c1-700 /tmp/b.json)" >> $O
