# DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 divergence bisection with the deterministic mode (4/4 divergent on the dp path)
mkdir -p gpurun_out
OUT=gpurun_out/pc_bisect.log
: > $OUT
run() {  # label, bench args, env...
  local label=$1 args=$2; shift 2
  for i in 1 2; do
    env DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 HCB_DETERMINISTIC=1 HCB_BENCH_LOSS_TRACE=1 "$@" timeout -k 10 200 python bench.py --steps 8 --warmup 5 $args > gpurun_out/v.log 2>&1 || exit 1
    echo "$label: $(grep losses gpurun_out/v.log | cut -c1-90)" >> $OUT
  done
}
run "single (no fork)" ""
run "dp, collectives skipped" "--force_dp_path" HCB_COMM_SKIP_RCCL=1
run "dp, no overlap (one fork after backward)" "--force_dp_path" HCB_OVERLAP=0
run "dp, one segment" "--force_dp_path" HCB_SEGMENT_PARAMS=1000000000
run "dp, no graph pool reuse" "--force_dp_path" PYTORCH_NO_CUDA_MEMORY_CACHING=1
cat $OUT
