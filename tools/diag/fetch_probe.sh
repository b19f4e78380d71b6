#!/bin/bash
# HBM bytes of one memory-bound stage-1 plane GEMM per cfg (rocprofv3 --pmc FETCH_SIZE WRITE_SIZE: 3 + 2 TCC
# counters would exceed 4, so one pass each)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/r6x; mkdir -p $O
L=${L:-stage1/block2/conv1}; OP=${OP:-fwd}
for c in ${CFGS:-16 20 4 19}; do
  P="python $R/tools/layer_probe.py --fp32 --layer $L --op $OP --cfg $c --reps 20"
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/f$c -o run -- $P > $O/f$c.log 2>&1) || exit 2
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/w$c -o run -- $P > $O/w$c.log 2>&1) || exit 3
  grep -v amdgpu.ids $O/f$c.log | tail -1
  python - "$O/f$c" "$O/w$c" <<'PY'
import csv, glob, sys, statistics
def val(d, name):
    f = glob.glob(d + "/**/run_counter_collection.csv", recursive=True)[0]
    per = {}
    for r in csv.DictReader(open(f)):
        if "conv" in r["Kernel_Name"] and r["Counter_Name"] == name:
            per.setdefault(r["Dispatch_Id"], 0.0)
            per[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return statistics.median(per.values()), len(per)
fs, n = val(sys.argv[1], "FETCH_SIZE"); ws, _ = val(sys.argv[2], "WRITE_SIZE")
print(f"   FETCH {fs / 1024:.1f} MB  WRITE {ws / 1024:.1f} MB per launch (median of {n}; counters in KB)")
PY
done
