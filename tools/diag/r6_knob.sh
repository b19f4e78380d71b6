#!/bin/bash
# in-step A/B of the persistent BNB epilogue (knob p3p_bnb 0 vs 1) and the interleaved A/A bands
set -o pipefail
O=gpurun_out/r6m
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp32_native_gpu.py \
  -k "persistent_fused or fused_bn_backward" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 420 python -u tools/step_tune.py --dtype fp32 --knob_ab p3p_bnb:0:1 --rounds 2 --aa_reps 4 --reps 20 \
  > $O/knob_fp32.txt 2>&1 || { tail -20 $O/knob_fp32.txt; exit 1; }
grep step_tune $O/knob_fp32.txt
timeout -k 10 420 python -u tools/step_tune.py --dtype bf16 --aa_only --rounds 2 --aa_reps 4 --reps 20 \
  > $O/aa_bf16.txt 2>&1 || { tail -20 $O/aa_bf16.txt; exit 1; }
grep step_tune $O/aa_bf16.txt
