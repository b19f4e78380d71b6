mkdir -p gpurun_out
timeout -k 10 100 python -u tools/diag_bn_stats.py > gpurun_out/diag_final.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_bn_shift_gpu.py -m gpu -x -q -s --timeout 120 --timeout-method thread > gpurun_out/t_shift3.log 2>&1 &&
for s in 1 0 1 0; do HCB_BN_SHIFT=$s timeout -k 10 200 python bench.py --steps 60 --warmup 10 > gpurun_out/bv.json 2>/dev/null || exit 1; echo "HCB_BN_SHIFT=$s $(cut -c1-160 gpurun_out/bv.json)" >> gpurun_out/bench_shift.log; done &&
for pc in 1 0 1; do DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc timeout -k 10 120 tools/graph_fork_repro 3000 >> gpurun_out/graph_repro.log 2>&1 || { echo "repro rc=$?" >> gpurun_out/graph_repro.log; }; done &&
bash tools/dp_variants.sh DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 > gpurun_out/dpv_nopk.log 2>&1 &&
HCB_KERNELS_SO=abvar/pk/_hcb_kernels.so bash tools/dp_variants.sh DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 > gpurun_out/dpv_pk.log 2>&1
