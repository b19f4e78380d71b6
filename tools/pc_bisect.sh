#!/bin/bash
# GPU: DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 divergence bisection (tools/pc_bisect.py), two runs per
# variant; one JSON line per run in gpurun_out/pc_bisect.log
mkdir -p gpurun_out
OUT=gpurun_out/pc_bisect.log
: > $OUT
run() {  # label, args...
  local label=$1; shift
  for i in 1 2; do
    DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 240 python tools/pc_bisect.py "$@" > gpurun_out/pcb.json 2> gpurun_out/pcb.err || { echo "$label: run failed"; tail -20 gpurun_out/pcb.err; exit 1; }
    echo "$label | $(cut -c1-400 gpurun_out/pcb.json)" | tee -a $OUT
  done
}
run "A bench-like"            --tune --lr sched --trace
run "B bench-like, no trace"  --tune --lr sched
run "C no tune"               --lr sched --trace
run "D const lr"              --tune --trace
run "E sync each replay"      --tune --lr sched --trace --sync_each
run "F single graph (no fork)" --tune --lr sched --trace --single
run "G race-like"             --lr const --graph_warmup 1 --clone --seed 5
