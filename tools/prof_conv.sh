#!/bin/bash
# Kernel-level counter study of single conv problems (run on the GPU box via gpurun).
#   LAYERS="stage3/block1/conv2:fwd:4 ..." bash tools/prof_conv.sh
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
python __graft_entry__.py > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
rocprofv3 --list-avail > gpurun_out/pmc/avail.txt 2>&1 || true
timeout -k 10 300 python tools/gemm_ref.py > gpurun_out/gemm_ref.log 2>&1 || { echo gemm_ref failed; tail gpurun_out/gemm_ref.log; exit 1; }
grep -v '^{' gpurun_out/gemm_ref.log
SETS=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS")
for spec in ${LAYERS:-stage3/block1/conv2:fwd:4 stage3/block1/conv2:fwd:0}; do
  IFS=: read layer pass cfg <<< "$spec"
  tag=$(echo "$layer-$pass-$cfg" | tr '/' '_')
  timeout -k 10 120 python tools/conv_micro.py --layer $layer --pass $pass --cfg $cfg --reps 20 || exit 1
  i=0
  for set in "${SETS[@]}"; do
    cd /tmp && timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmc/$tag.$i -o run -- python $R/tools/conv_micro.py --layer $layer --pass $pass --cfg $cfg --reps 5 > $R/gpurun_out/pmc/$tag.$i.log 2>&1 || { echo "pmc failed $tag $i"; tail -5 $R/gpurun_out/pmc/$tag.$i.log; exit 1; }
    cd $R
    i=$((i+1))
  done
done
echo "prof_conv done"
