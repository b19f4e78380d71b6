# tuner timing fidelity: retune resnet50 with per-launch isolated timing (autotune.TUNE_ISOLATE), then a
# same-box A/B of the resulting cache against the current one
set -o pipefail
mkdir -p gpurun_out
T=azure_hc_intel_tf_amd/tuned
cp $T/mi355x.json /tmp/cache_cur.json
HCB_TUNE_REPS=15 timeout -k 10 900 python -u -c "import sys; sys.argv=['x','resnet50']; sys.path.insert(0,'tools'); from azure_hc_intel_tf_amd.ops import autotune; autotune.TUNE_ISOLATE=True; import retune_conv; retune_conv.main()" > gpurun_out/r3y_tune.log 2>&1 || exit 1
cp $T/mi355x.json /tmp/cache_iso.json
cp /tmp/cache_iso.json gpurun_out/r3y_cache_iso.json
O=gpurun_out/r3y_ab.txt
: > $O
for r in 1 2 3; do for v in cur iso; do
  cp /tmp/cache_$v.json $T/mi355x.json
  timeout -k 10 300 python bench.py --steps 40 --warmup 10 > /tmp/b.json || exit 1
  echo "bench $v: $(python -c "import json;d=json.load(open('/tmp/b.json'));print(d['value'], d['ms_per_step'])")" >> $O
done; done
