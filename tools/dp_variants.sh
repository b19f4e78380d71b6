# Repeat the forced multi-GPU step path on one GPU (device-side loss trace) under env variants.
#   BENCH_ARGS="--compression bf16" bash tools/dp_variants.sh "HCB_X=1" "HCB_COMM_WATCHDOG=0" ...
mkdir -p gpurun_out
run() { echo "== $* $BENCH_ARGS"; env HCB_BENCH_LOSS_TRACE=1 "$@" timeout -k 10 200 python bench.py --steps 8 --warmup 5 --force_dp_path $BENCH_ARGS > gpurun_out/v.log 2>&1 || { tail -5 gpurun_out/v.log; return 1; }; grep "losses" gpurun_out/v.log | cut -c1-120; }
for v in "$@"; do run $v || exit 1; done
