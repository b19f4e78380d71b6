#!/bin/bash
# the stem GEMM per cfg: time, then L2 request counters (one rocprofv3 --pmc pass per cfg)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/r6st; mkdir -p $O
timeout -k 10 120 python tools/diag/stem_gemm_probe.py > $O/time.txt 2>&1 || { tail -20 $O/time.txt; exit 1; }
grep -v amdgpu.ids $O/time.txt
for c in 19 34; do
  P="python $R/tools/diag/stem_gemm_probe.py --cfgs $c --reps 20"
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum \
    --kernel-trace --output-format csv -d $O/p$c -o run -- $P > $O/p$c.log 2>&1) || exit 2
  python tools/pmc_table.py $O/p$c conv
done
