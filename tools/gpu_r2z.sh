# data-parallel path rehearsal on one GPU with the current kernels: forced DP step (1-rank RCCL engine,
# collectives captured in the step graph) and a 2-rank gloo run sharing the GPU
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --force_dp_path --steps 30 --warmup 10 > gpurun_out/z_dp.json 2> gpurun_out/z_dp.err || { tail -20 gpurun_out/z_dp.err; exit 1; }
cut -c1-400 gpurun_out/z_dp.json
HCB_BENCH_ONE_DEVICE=1 HCB_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/z_gloo2.json 2> gpurun_out/z_gloo2.err || { tail -20 gpurun_out/z_gloo2.err; exit 1; }
cut -c1-400 gpurun_out/z_gloo2.json
grep -i "total images/sec" gpurun_out/z_gloo2.err | head -4
