#!/bin/bash
# Packet-capture memset check (tools/graph_fork_repro.hip modes 10 / 11 / 6), capture on and off.
# A run that finds wrong values exits 1 and the script goes on; any other failure (time limit,
# abort, fault) ends it.
cd "$(dirname "$0")/.."
for m in ${MODES:-10 11 6}; do
  for pc in 1 0; do
    DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc timeout -k 10 60 ./tools/graph_fork_repro ${REPLAYS:-200} $m
    rc=$?
    if [ $rc -gt 1 ]; then echo "graph_fork_repro mode $m pc $pc: rc=$rc -- stopping"; exit $rc; fi
  done
done
