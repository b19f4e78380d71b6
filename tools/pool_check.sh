set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_stem_pool_bwd_gpu.py tests/test_fp32_native_gpu.py tests/test_race_gpu.py > gpurun_out/pool_tests.log 2>&1; rc=$?; tail -3 gpurun_out/pool_tests.log; [ $rc -eq 0 ] || exit 1
TAG=r4pool bash tools/gpu_run.sh bench prof:--compute_dtype,bf16,--secondary,none,--steps,10,--warmup,3
