#!/bin/bash
# A/B of the BN statistic replica count (HCB_STAT_R) on ResNet-50 bs=64, one box, back to back.
set -o pipefail
mkdir -p gpurun_out
for v in 8 16 32 4 8; do
  HCB_STAT_R=$v timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/abr_$v.log 2>&1 || { tail -20 gpurun_out/abr_$v.log; exit 1; }
  echo "STAT_R=$v $(tail -1 gpurun_out/abr_$v.log | cut -c1-200)"
done
