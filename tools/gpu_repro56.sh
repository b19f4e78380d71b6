# graph_fork_repro memset modes (5: forks + memset nodes, 6: memset nodes, no forks), packet capture on / off
mkdir -p gpurun_out
: > gpurun_out/repro56.log
for m in 5 6 5 6; do for pc in 1 0; do
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc timeout -k 10 120 tools/graph_fork_repro 2000 $m >> gpurun_out/repro56.log 2>&1
  rc=$?
  [ $rc -eq 0 ] || echo "mode $m pc $pc rc=$rc" >> gpurun_out/repro56.log
  [ $rc -le 1 ] || exit $rc   # a fault / timeout: start nothing more
done; done
cat gpurun_out/repro56.log
