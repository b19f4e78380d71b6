set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/r3j_pc.log
: > $OUT
for mode in 0 1 5 6 7 8 9; do
  for pc in 1 0; do
    DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc timeout -k 10 120 tools/graph_fork_repro 2000 $mode >> $OUT 2>&1
    rc=$?
    [ $rc -gt 1 ] && { echo "repro mode $mode pc $pc: rc $rc"; exit 1; }
  done
done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 600 python -u tools/pc_race_bisect.py single >> $OUT 2>&1
