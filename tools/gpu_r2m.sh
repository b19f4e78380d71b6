# stride-phase data gradients: tests, then inception3 / resnet50_v1.5 / resnet50 A/B
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dgrad_phases_gpu.py tests/test_kernels_gpu.py tests/test_zoo_gpu.py tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_phase.log 2>&1 || { tail -40 gpurun_out/t_phase.log; exit 1; }
tail -2 gpurun_out/t_phase.log
: > gpurun_out/bench_phase.log
for spec in inception3:64 resnet50_v1.5:64 resnet50:64; do IFS=: read m b <<< "$spec"; for ph in 1 0; do
  HCB_DGRAD_PHASES=$ph timeout -k 10 300 python bench.py --model $m --batch_size $b --steps 30 --warmup 8 > gpurun_out/bv.json 2>/dev/null || exit 1
  echo "$m HCB_DGRAD_PHASES=$ph $(python -c 'import json;d=json.load(open("gpurun_out/bv.json"));print(d["value"], d["ms_per_step"])')" >> gpurun_out/bench_phase.log
done; done
cat gpurun_out/bench_phase.log
