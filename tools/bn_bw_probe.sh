#!/bin/bash
# BN streaming-pass throughput vs a plain copy (tools/bn_bw_probe.py) inside a replayed graph, at the
# default grid and at VARIANTS="<HCB_BN_BLOCKS>:<HCB_BN_RPT> ..." grids. Output: gpurun_out/bnbw.log
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/bnbw.log
: > $O
timeout -k 10 120 python tools/bn_bw_probe.py --graph >> $O 2>&1 || exit 1
for v in ${VARIANTS:-1000000:1 1000000:2 8192:1 4096:2}; do
  IFS=: read b r <<< "$v"
  echo "== blocks $b rows/thread $r" >> $O
  HCB_BN_BLOCKS=$b HCB_BN_RPT=$r timeout -k 10 120 python tools/bn_bw_probe.py --graph >> $O 2>&1 || exit 1
done
