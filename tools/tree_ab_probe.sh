#!/bin/bash
# tools/bn_bw_probe.py --graph from ./abbase (baseline) and from the working tree, then tools/tree_ab.sh.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
(cd $R/abbase && timeout -k 10 120 python tools/bn_bw_probe.py --graph > $R/gpurun_out/probe_base.log 2>&1) &&
timeout -k 10 120 python tools/bn_bw_probe.py --graph > gpurun_out/probe_new.log 2>&1 &&
paste <(grep -v amdgpu.ids gpurun_out/probe_base.log | sed -n 2,11p | cut -c1-80) <(grep -v amdgpu.ids gpurun_out/probe_new.log | sed -n 2,11p | cut -c22-80) &&
bash tools/tree_ab.sh
