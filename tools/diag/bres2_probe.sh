#!/bin/bash
# B-resident persistent plane GEMM over several N tiles (cfg 31-36): fp64 tests, isolated timings
set -o pipefail
O=gpurun_out/r6zg; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp32_native_gpu.py \
  -k "short_k_gemm or (fwd_dgrad_wgrad_match_fp64 and (31 or 32 or 33 or 34 or 35 or 36))" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for spec in "stage3/block2/conv3 17 18 22 33 34 35" "stage2/block2/conv3 19 36 34 35 32" "stage1/block1/conv3 18 32"; do
  set -- $spec; L=$1; shift
  for c in "$@"; do
    timeout -k 10 60 python tools/layer_probe.py --fp32 --layer $L --op fwd --cfg $c --reps 50 2>&1 | grep -v amdgpu.ids >> $O/probe.txt || exit 1
  done
done
cat $O/probe.txt
