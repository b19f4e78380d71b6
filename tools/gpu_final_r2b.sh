# round-2 final run (second session): smoke, whole GPU suite, default bench, kernel stats, README numbers
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/fc_smoke.log 2>&1 || { tail -20 gpurun_out/fc_smoke.log; exit 1; }
tail -1 gpurun_out/fc_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/fc_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/fc_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/fc_pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/fc_bench_default.json 2> gpurun_out/fc_bench_default.err || { tail -20 gpurun_out/fc_bench_default.err; exit 1; }
cut -c1-200 gpurun_out/fc_bench_default.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/fc_prof" -o run -- python "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/fc_prof.log" 2>&1 || { echo "rocprof failed"; exit 1; }
cd "$GRAFT_REPO_ROOT" && echo "prof done"
timeout -k 10 300 python bench.py --use_fp16 --steps 40 --warmup 10 > gpurun_out/fc_bench_fp16.json 2> gpurun_out/fc_bench_fp16.err || { tail -20 gpurun_out/fc_bench_fp16.err; exit 1; }
cut -c1-200 gpurun_out/fc_bench_fp16.json
bash tools/gpu_readme_numbers.sh
