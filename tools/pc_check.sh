#!/bin/bash
# GPU: does the graph-packet-capture divergence (profiles/r2f_graph_packet_capture.txt, section 4:
# bench.py --force_dp_path, deterministic, DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 -> inf/nan 4 of 4)
# still reproduce? The round-2 reproducer verbatim, 4 runs, then the default (atomic) mode, the
# compressed wire and the real-rank race detector, all with packet capture ON.
mkdir -p gpurun_out
OUT=gpurun_out/pc_check.log
: > $OUT
run() {  # label, env..., -- bench args
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 HCB_BENCH_LOSS_TRACE=1 "${envs[@]}" timeout -k 10 240 \
    python bench.py --steps 8 --warmup 5 "$@" > gpurun_out/pcc.log 2>&1 || { echo "$label: failed"; tail -20 gpurun_out/pcc.log; exit 1; }
  echo "$label | $(grep '\[bench\] losses' gpurun_out/pcc.log | cut -c1-150)" | tee -a $OUT
}
for i in 1 2 3 4; do run "det dp $i" HCB_DETERMINISTIC=1 -- --force_dp_path; done
for i in 1 2; do run "atomic dp $i" HCB_BENCH_X=0 -- --force_dp_path; done
run "det dp bf16 wire" HCB_DETERMINISTIC=1 -- --force_dp_path --compression bf16
run "det single" HCB_DETERMINISTIC=1 --
run "det dp block segments" HCB_DETERMINISTIC=1 -- --force_dp_path --backward_segments block
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 600 python -u -m pytest tests/test_race_gpu.py tests/test_comm_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/pcc_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pcc_tests.log; exit 1; }
echo "race + comm tests with packet capture on: $(tail -1 gpurun_out/pcc_tests.log)" | tee -a $OUT
