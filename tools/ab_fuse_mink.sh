set -o pipefail
mkdir -p gpurun_out
for v in 0 128 256 0; do
  HCB_FUSE_BN_BWD_MIN_K=$v timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/ab_$v.log 2>&1 || { tail -20 gpurun_out/ab_$v.log; exit 1; }
  echo "MIN_K=$v $(tail -1 gpurun_out/ab_$v.log | cut -c1-200)"
done
