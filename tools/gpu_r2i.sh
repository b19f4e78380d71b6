# native IEEE-fp16 kernel build: tests, then the full GPU suite, then --use_fp16 throughput
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fp16_native_gpu.py tests/test_precision_modes_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_fp16.log 2>&1 || { tail -40 gpurun_out/t_fp16.log; exit 1; }
tail -3 gpurun_out/t_fp16.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
timeout -k 10 200 python bench.py --use_fp16 --steps 40 --warmup 10 > gpurun_out/b_fp16.json 2> gpurun_out/b_fp16.err || { tail -20 gpurun_out/b_fp16.err; exit 1; }
cut -c1-300 gpurun_out/b_fp16.json
timeout -k 10 400 python tf_cnn_benchmarks.py --model=resnet152 --batch_size=128 --num_batches=30 --num_warmup_batches=10 --display_every=10 --optimizer=momentum --variable_update=horovod --use_fp16 --fp16_enable_auto_loss_scale --device=gpu > gpurun_out/c5_fp16.log 2>&1 || { tail -20 gpurun_out/c5_fp16.log; exit 1; }
grep -E "Precision|total images/sec|loss" gpurun_out/c5_fp16.log | tail -5
