set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "bn or fused" tests/test_fused_resbn_gpu.py tests/test_stem_pool_bwd_gpu.py tests/test_fp32_native_gpu.py tests/test_race_gpu.py > gpurun_out/bnc_tests.log 2>&1 && tail -2 gpurun_out/bnc_tests.log &&
VARIANTS=" " timeout -k 10 200 bash tools/bn_bw_probe.sh && grep -v amdgpu.ids gpurun_out/bnbw.log | head -12
