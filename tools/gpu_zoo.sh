mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_zoo_gpu.py tests/test_model_gpu.py > gpurun_out/zoo_gpu.log 2>&1 || { tail -30 gpurun_out/zoo_gpu.log; exit 1; }
tail -2 gpurun_out/zoo_gpu.log
for spec in ${MODELS:-resnet50_v2:64 vgg16:64 googlenet:128 alexnet:512 overfeat:128}; do
  IFS=: read m b <<< "$spec"
  timeout -k 10 600 python bench.py --model $m --batch_size $b --steps 20 --warmup 5 > gpurun_out/bench_$m.log 2>&1 || { echo "bench $m failed"; tail -20 gpurun_out/bench_$m.log; exit 1; }
  tail -1 gpurun_out/bench_$m.log | cut -c1-220
done
cp azure_hc_intel_tf_amd/tuned/mi355x.json gpurun_out/tuned_mi355x.json
