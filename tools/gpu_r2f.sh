# DEBUG_CLR_GRAPH_PACKET_CAPTURE investigation: minimal fork/join graphs vs the training step
mkdir -p gpurun_out
OUT=gpurun_out/packet_capture2.log
: > $OUT
for m in 1 2 3 4; do
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 120 tools/graph_fork_repro 2000 $m >> $OUT 2>&1 || echo "repro mode $m rc=$?" >> $OUT
done
dp() {  # label, env...
  local label=$1; shift
  for i in 1 2 3; do
    env DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 HCB_BENCH_LOSS_TRACE=1 "$@" timeout -k 10 200 python bench.py --steps 8 --warmup 5 --force_dp_path > gpurun_out/v.log 2>&1 || exit 1
    echo "$label $(grep losses gpurun_out/v.log | cut -c1-100)" >> $OUT
  done
}
dp "skip_rccl+no_watchdog" HCB_COMM_SKIP_RCCL=1 HCB_COMM_WATCHDOG=0
dp "comm_noop(no fork)" HCB_COMM_NOOP=1
dp "skip_rccl+no_overlap" HCB_COMM_SKIP_RCCL=1 HCB_OVERLAP=0
timeout -k 10 100 python -u tools/diag_bn_stats.py 2>&1 | grep "R=8" >> $OUT
for s in 1 0 1 0; do HCB_BN_SHIFT=$s timeout -k 10 200 python bench.py --steps 60 --warmup 10 > gpurun_out/bv.json 2>/dev/null || exit 1; echo "HCB_BN_SHIFT=$s $(cut -c1-160 gpurun_out/bv.json)" >> $OUT; done
