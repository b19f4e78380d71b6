# Effective clock of one conv GEMM launch (tools/layer_probe.py), cfg A vs cfg B: rocprofv3 --pmc
# GRBM_GUI_ACTIVE (summed over the 8 XCDs) with the kernel trace; clock = GUI_ACTIVE / 8 / duration
# (MI355X guide, DVFS give-back). Args: LAYER OP CFG_A CFG_B [ENV_B]
set -o pipefail
L=$1; OP=$2; A=$3; B=$4; EB=${5:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp
for v in A B; do
  if [ $v = A ]; then c=$A; e=""; else c=$B; e="$EB"; fi
  d=$R/gpurun_out/dvfs_${v}
  rm -rf $d
  env $e timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $d -o run \
    -- python $R/tools/layer_probe.py --fp32 --layer $L --op $OP --reps 40 --cfg $c > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  python $R/tools/diag/dvfs_summary.py $d "$v cfg=$c $e"
done
