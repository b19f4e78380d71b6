# sanity of the exact final tree: smoke, whole GPU suite, default bench
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/fd_smoke.log 2>&1 || { tail -20 gpurun_out/fd_smoke.log; exit 1; }
tail -1 gpurun_out/fd_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fd_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/fd_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/fd_pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/fd_bench.json 2> gpurun_out/fd_bench.err || { tail -20 gpurun_out/fd_bench.err; exit 1; }
cut -c1-220 gpurun_out/fd_bench.json
