#!/bin/bash
# Kernel-level counter study of single conv problems (run on the GPU box via gpurun).
#   LAYERS="stage3/block1/conv2:fwd:4 ..." bash tools/prof_conv.sh
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
[ "${LIST:-0}" = "1" ] && { rocprofv3 --list-avail > gpurun_out/pmc/avail.txt 2>&1 || true; }
SETS=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum")
for spec in ${LAYERS:-stage3/block1/conv2:fwd:4 stage3/block1/conv2:fwd:0}; do
  IFS=: read layer pass cfg splits <<< "$spec"
  SPL=""; [ -n "$splits" ] && SPL="--splits $splits"
  tag=$(echo "$layer-$pass-$cfg-$splits" | tr '/' '_')
  timeout -k 10 120 python tools/conv_micro.py --layer $layer --pass $pass --cfg $cfg $SPL --reps 20 || exit 1
  i=0
  for set in "${SETS[@]}"; do
    cd /tmp && timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmc/$tag.$i -o run -- python $R/tools/conv_micro.py --layer $layer --pass $pass --cfg $cfg $SPL --reps 5 > $R/gpurun_out/pmc/$tag.$i.log 2>&1 || { echo "pmc failed $tag $i"; tail -5 $R/gpurun_out/pmc/$tag.$i.log; exit 1; }
    cd $R
    i=$((i+1))
  done
done
echo "prof_conv done"
