# fused projection-shortcut BN: tests, then bench A/B
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_fused_resbn_gpu.py tests/test_model_gpu.py tests/test_determinism_gpu.py tests/test_fp16_native_gpu.py tests/test_bn_shift_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_resbn.log 2>&1 || { tail -40 gpurun_out/t_resbn.log; exit 1; }
tail -2 gpurun_out/t_resbn.log
: > gpurun_out/bench_resbn.log
for f in 1 0 1 0; do HCB_FUSE_RES_BN=$f timeout -k 10 200 python bench.py --steps 60 --warmup 10 > gpurun_out/bv.json 2>/dev/null || exit 1; echo "HCB_FUSE_RES_BN=$f $(cut -c1-150 gpurun_out/bv.json)" >> gpurun_out/bench_resbn.log; done
cat gpurun_out/bench_resbn.log
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof3" -o run -- python "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/prof3.log" 2>&1 || { echo "rocprof failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof3.log"; exit 1; }
cd $GRAFT_REPO_ROOT && grep metric gpurun_out/prof3.log | cut -c1-150
