# A/B an environment knob on the default bench: bash tools/gpu_ab_env.sh VAR "a b" [reps]
mkdir -p gpurun_out
VAR=$1; VALS=$2; REPS=${3:-2}
OUT=gpurun_out/ab_$VAR.log
: > $OUT
for r in $(seq $REPS); do for v in $VALS; do
  env $VAR=$v timeout -k 10 200 python bench.py --steps 60 --warmup 10 > gpurun_out/bv.json 2>/dev/null || exit 1
  echo "$VAR=$v $(python -c 'import json;d=json.load(open("gpurun_out/bv.json"));print(d["value"], d["ms_per_step"])')" >> $OUT
done; done
cat $OUT
