# careful retune of the headline config (resnet50 bs64, 20 timed launches per candidate): fwd/dgrad + wgrad, bench A/B
mkdir -p gpurun_out
export TMPDIR=/tmp
cp azure_hc_intel_tf_amd/tuned/mi355x.json gpurun_out/ad_cache_before.json
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/ad_b.json 2> gpurun_out/ad_b.err || { tail -20 gpurun_out/ad_b.err; exit 1; }
  echo "bench (reps-5 cache) $(python -c 'import json;d=json.load(open("gpurun_out/ad_b.json"));print(d["value"], d["ms_per_step"])')"
done
HCB_TUNE_REPS=20 timeout -k 10 600 python -u tools/retune_conv.py resnet50 > gpurun_out/ad_retune_conv.log 2>&1 || { tail -20 gpurun_out/ad_retune_conv.log; exit 1; }
HCB_TUNE_REPS=20 timeout -k 10 600 python -u tools/retune_wgrad.py resnet50 > gpurun_out/ad_retune_wgrad.log 2>&1 || { tail -20 gpurun_out/ad_retune_wgrad.log; exit 1; }
grep "tuned [0-9]* problems" gpurun_out/ad_retune_conv.log gpurun_out/ad_retune_wgrad.log
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/ad_b.json 2> gpurun_out/ad_b.err || { tail -20 gpurun_out/ad_b.err; exit 1; }
  echo "bench (reps-20 retune) $(python -c 'import json;d=json.load(open("gpurun_out/ad_b.json"));print(d["value"], d["ms_per_step"])')"
done
