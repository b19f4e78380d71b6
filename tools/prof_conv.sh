#!/bin/bash
# Kernel-level hardware-counter study of single conv problems (run on the GPU box via gpurun).
#   LAYERS="stage3/block1/conv2:fwd:- stage3/block1/conv2:fwd:4 ..." bash tools/prof_conv.sh
# spec = layer:pass:cfg[:splits]; cfg "-" = the autotuned config. One rocprofv3 pass per
# counter set (at most 8 SQ / 4 TCC counters per pass), each under its own hard time limit.
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
SETS=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
      "FETCH_SIZE"
      "TCC_HIT_sum TCC_MISS_sum WRITE_SIZE")
for spec in ${LAYERS:-stage3/block1/conv2:fwd:-}; do
  IFS=: read layer pass cfg splits <<< "$spec"
  ARGS="--layer $layer --pass $pass"
  [ "$cfg" != "-" ] && ARGS="$ARGS --cfg $cfg"
  [ -n "$splits" ] && ARGS="$ARGS --splits $splits"
  tag=$(echo "$layer-$pass-$cfg-$splits" | tr '/' '_')
  timeout -k 10 120 python tools/conv_micro.py $ARGS --reps 20 || exit 1
  i=0
  for set in "${SETS[@]}"; do
    cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmc/$tag.$i -o run -- python $R/tools/conv_micro.py $ARGS --reps 5 > $R/gpurun_out/pmc/$tag.$i.log 2>&1 || { echo "pmc failed $tag $i"; tail -5 $R/gpurun_out/pmc/$tag.$i.log; exit 1; }
    cd $R
    i=$((i+1))
  done
done
echo "prof_conv done"
