#!/bin/bash
# GPU: graph_fork_repro cross-XCD modes (7, 8) and the no-fork memset chain (6), with and without
# graph packet capture; one line each in gpurun_out/pc_xcd.log
mkdir -p gpurun_out
OUT=gpurun_out/pc_xcd.log
: > $OUT
for mode in 6 7 8; do
  for pc in 1 0; do
    DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc timeout -k 10 120 tools/graph_fork_repro 2000 $mode >> $OUT 2>&1
    rc=$?
    [ $rc -gt 1 ] && { echo "repro mode $mode pc $pc: rc $rc"; cat $OUT; exit 1; }
  done
done
cat $OUT
