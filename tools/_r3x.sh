# same-box A/B of two autotune caches: r3k (before the KU=2 configs) vs r3w (KU=2 configs chosen)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3x_ab.txt
: > $O
T=azure_hc_intel_tf_amd/tuned
for r in 1 2 3; do for v in r3k ku2; do
  cp $T/mi355x_$v.json $T/mi355x.json
  timeout -k 10 300 python bench.py --steps 40 --warmup 10 > /tmp/b.json || exit 1
  echo "bench $v: $(python -c "import json;d=json.load(open('/tmp/b.json'));print(d['value'], d['ms_per_step'])")" >> $O
done; done
