#!/bin/bash
# BN-kernel tests, then the same-box bench A/B against ./abbase (tools/tree_ab.sh).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "bn or fused" \
  tests/test_fused_resbn_gpu.py tests/test_stem_pool_bwd_gpu.py tests/test_fp32_native_gpu.py tests/test_race_gpu.py \
  tests/test_determinism_gpu.py > gpurun_out/bnab_tests.log 2>&1 && tail -1 gpurun_out/bnab_tests.log &&
ROUNDS=${ROUNDS:-3} bash tools/tree_ab.sh
