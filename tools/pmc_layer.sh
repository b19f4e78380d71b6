#!/bin/bash
# Hardware counters of ONE conv GEMM (tools/layer_probe.py), two rocprofv3 --pmc passes of their own:
#   LAYERS="stage3/block1/conv2:fwd stage3/block1/conv2:wgrad" TAG=r4s bash tools/pmc_layer.sh [--fp32]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
for lo in ${LAYERS:-stage3/block1/conv2:fwd}; do
  layer=${lo%%:*}; op=${lo##*:}
  O=$R/gpurun_out/${TAG:-pmc}_$(echo $layer | tr / _)_$op
  P="python $R/tools/layer_probe.py $* --layer $layer --op $op --reps 30"
  timeout -k 10 120 $P > ${O}_time.txt 2>&1 || exit 1
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS \
    --kernel-trace --output-format csv -d ${O}_pmc1 -o run -- $P > ${O}_pmc1.log 2>&1) || exit 2
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum \
    --kernel-trace --output-format csv -d ${O}_pmc2 -o run -- $P > ${O}_pmc2.log 2>&1) || exit 3
  { cat ${O}_time.txt | grep -v amdgpu.ids; python tools/pmc_table.py ${O}_pmc1 conv; python tools/pmc_table.py ${O}_pmc2 conv; } \
    > ${O}_pmc.txt
  cat ${O}_pmc.txt
done
