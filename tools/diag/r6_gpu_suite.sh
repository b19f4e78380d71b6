#!/bin/bash
# the whole GPU test tier in one pytest process, then smoke()
set -o pipefail
O=gpurun_out/${TAG:-r6n}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $O/gpu_tests.txt 2>&1
rc=$?
grep -E "passed|failed" $O/gpu_tests.txt | tail -3
grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -4 $O/smoke.txt
exit $rc
