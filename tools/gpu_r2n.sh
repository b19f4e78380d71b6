mkdir -p gpurun_out
timeout -k 10 600 python -u tools/tune_all.py inception3 resnet50_v1.5 > gpurun_out/tune_phase.log 2>&1 || { tail -20 gpurun_out/tune_phase.log; exit 1; }
grep -v "  tuned" gpurun_out/tune_phase.log | tail -3
: > gpurun_out/bench_phase2.log
for spec in inception3:64 resnet50_v1.5:64; do IFS=: read m b <<< "$spec"; for ph in 1 0 1 0; do
  HCB_DGRAD_PHASES=$ph timeout -k 10 300 python bench.py --model $m --batch_size $b --steps 30 --warmup 8 > gpurun_out/bv.json 2>/dev/null || exit 1
  echo "$m HCB_DGRAD_PHASES=$ph $(python -c 'import json;d=json.load(open("gpurun_out/bv.json"));print(d["value"], d["ms_per_step"])')" >> gpurun_out/bench_phase2.log
done; done
cat gpurun_out/bench_phase2.log
