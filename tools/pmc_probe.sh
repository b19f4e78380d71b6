set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r4n
P="python $R/tools/layer_probe.py --fp32 --layer stage3/block1/conv2 --op fwd --reps 30"
timeout -k 10 120 $P > ${O}_time.txt 2>&1 || exit 1
(cd /tmp && timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d ${O}_pmc1 -o run -- $P > ${O}_pmc1.log 2>&1) || exit 2
(cd /tmp && timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum --kernel-trace --output-format csv -d ${O}_pmc2 -o run -- $P > ${O}_pmc2.log 2>&1) || exit 3
python tools/pmc_table.py ${O}_pmc1 p3 > ${O}_pmc.txt; python tools/pmc_table.py ${O}_pmc2 p3 >> ${O}_pmc.txt
echo done
