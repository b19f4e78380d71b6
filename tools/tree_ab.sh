#!/bin/bash
# Same-box A/B of the working tree against a baseline copy of the package in ./abbase (bench.py +
# azure_hc_intel_tf_amd/ built from an earlier commit; git-ignored). Alternates the two, ROUNDS times.
# Output: gpurun_out/tree_ab.log
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/tree_ab.log
: > $O
for r in $(seq ${ROUNDS:-2}); do
  for arm in base new; do
    d=$R; [ $arm = base ] && d=$R/abbase
    (cd $d && timeout -k 10 400 python bench.py --steps ${STEPS:-40} --warmup 10 ${BENCH_ARGS:-} > $R/gpurun_out/ab_$arm.json 2> $R/gpurun_out/ab_$arm.err) || { tail -20 $R/gpurun_out/ab_$arm.err; exit 1; }
    echo "$arm $(python -c "import json;d=json.load(open('$R/gpurun_out/ab_$arm.json'));print(d['value'], d['ms_per_step'], 'bf16', d.get('bf16_value'), d.get('bf16_ms_per_step'))")" | tee -a $O
  done
done
