#!/bin/bash
# B-resident persistent plane GEMM (cfg 31-34): fp64 tests, then isolated timings against the tuned plans
set -o pipefail
O=gpurun_out/r6y; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp32_native_gpu.py \
  -k "short_k_gemm" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for spec in "stage1/block1/conv3 18 31 32 19" "stage1/block1/shortcut 18 31 32" "stage1/block2/conv1 16 33 34 20" "stage1/block1/conv1 20 33 34"; do
  set -- $spec; L=$1; shift
  for c in "$@"; do
    timeout -k 10 60 python tools/layer_probe.py --fp32 --layer $L --op fwd --cfg $c --reps 50 2>&1 | grep -v amdgpu.ids >> $O/probe.txt || exit 1
  done
done
cat $O/probe.txt
