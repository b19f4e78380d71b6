#!/bin/bash
# GPU: packet-capture trigger bisection, part 2 -- the scalar-cache chain of graph_fork_repro
# (mode 9) and the race detector's single-graph run with module switches flipped
mkdir -p gpurun_out
for pc in 1 0; do
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc timeout -k 10 120 tools/graph_fork_repro 2000 9 | tee -a gpurun_out/pc_bisect2.log
  [ ${PIPESTATUS[0]} -gt 1 ] && exit 1
done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 900 python -u tools/pc_race_bisect.py single | tee -a gpurun_out/pc_bisect2.log
