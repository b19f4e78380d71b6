mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bn_probe.py > gpurun_out/r_bn_probe.txt 2>&1; rc=$?; cat gpurun_out/r_bn_probe.txt; [ $rc -eq 0 ] || exit $rc
for v in 4 1 2; do HCB_BN_ROWS_PER_THREAD=$v timeout -k 10 300 python -u tools/bn_probe.py > gpurun_out/r_bn_probe_$v.txt 2>&1 || exit 1; echo "rows/thread $v"; cat gpurun_out/r_bn_probe_$v.txt | grep -v amdgpu; done
