set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_stem_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/stem_tests.log 2>&1; rc=$?; tail -15 gpurun_out/stem_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_s2d.log 2>&1 || { tail -20 gpurun_out/bench_s2d.log; exit 1; }
grep -v amdgpu gpurun_out/bench_s2d.log
cp azure_hc_intel_tf_amd/tuned/mi355x.json gpurun_out/tuned_after.json
HCB_STEM_S2D=0 timeout -k 10 400 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_direct.log 2>&1 || { tail -20 gpurun_out/bench_direct.log; exit 1; }
grep -v amdgpu gpurun_out/bench_direct.log
timeout -k 10 400 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_s2d_b.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/bench_s2d_b.log
