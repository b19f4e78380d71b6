# isolated-timing retune WITH the KU=2 configs as candidates, A/B against the isolated-timing cache without them
set -o pipefail
mkdir -p gpurun_out
T=azure_hc_intel_tf_amd/tuned
cp gpurun_out/r3y_cache_iso.json /tmp/cache_iso.json
cp /tmp/cache_iso.json $T/mi355x.json
HCB_TUNE_REPS=15 timeout -k 10 900 python -u -c "import sys; sys.argv=['x','resnet50']; sys.path.insert(0,'tools'); from azure_hc_intel_tf_amd.ops import autotune, functional as Fn; autotune.TUNE_ISOLATE=True; Fn.TUNE_KU2=True; import retune_conv; retune_conv.main()" > gpurun_out/r3z_tune.log 2>&1 || exit 1
cp $T/mi355x.json /tmp/cache_ku2.json
cp /tmp/cache_ku2.json gpurun_out/r3z_cache_isoku2.json
O=gpurun_out/r3z_ab.txt
: > $O
for r in 1 2 3; do for v in iso ku2; do
  cp /tmp/cache_$v.json $T/mi355x.json
  timeout -k 10 300 python bench.py --steps 40 --warmup 10 > /tmp/b.json || exit 1
  echo "bench $v: $(python -c "import json;d=json.load(open('/tmp/b.json'));print(d['value'], d['ms_per_step'])")" >> $O
done; done
