# kernel-class profile of one model's bench step: bash tools/gpu_prof_model.sh MODEL BATCH
mkdir -p gpurun_out
export TMPDIR=/tmp
M=$1; B=$2
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$M" -o run -- python "$GRAFT_REPO_ROOT/bench.py" --model $M --batch_size $B --steps 10 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/prof_$M.log" 2>&1 || { echo "rocprof failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_$M.log"; exit 1; }
cd "$GRAFT_REPO_ROOT" && grep metric gpurun_out/prof_$M.log | cut -c1-150
