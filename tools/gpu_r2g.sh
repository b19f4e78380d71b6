# packet capture on + distinct fork/join events per edge (HCB_COMM_FRESH_EVENTS=1)
mkdir -p gpurun_out
OUT=gpurun_out/packet_capture3.log
: > $OUT
dp() {  # label, n, env...
  local label=$1 n=$2; shift 2
  for i in $(seq $n); do
    env DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 HCB_BENCH_LOSS_TRACE=1 "$@" timeout -k 10 200 python bench.py --steps 8 --warmup 5 --force_dp_path > gpurun_out/v.log 2>&1 || exit 1
    echo "$label $(grep losses gpurun_out/v.log | cut -c1-100)" >> $OUT
  done
}
dp "fresh_events" 5 HCB_COMM_FRESH_EVENTS=1
dp "fresh_events+skip_rccl" 3 HCB_COMM_FRESH_EVENTS=1 HCB_COMM_SKIP_RCCL=1
dp "shared_events(control)" 3
