#!/bin/bash
# One parametrised GPU-box runner (gpurun): every step is named on the command line and runs under
# its own time limit; the first failing step ends the script (no retries on the GPU).
#
#   gpurun -- bash tools/gpu_run.sh smoke tests bench prof
#   gpurun -- bash tools/gpu_run.sh tests:tests/test_kernels_gpu.py bench:--steps=30 prof:--steps=10
#   TAG=r3a gpurun -- bash tools/gpu_run.sh bench readme
#
# steps:
#   smoke            __graft_entry__.smoke()
#   tests[:files]    pytest -m gpu (whole suite, or the comma-separated files)
#   bench[:args]     python bench.py (args comma-separated, e.g. bench:--batch_size=256)
#   benchab:ENV      bench.py with and without ENV (e.g. benchab:HCB_X=0), interleaved 2 rounds
#   convab:DIR       tools/conv_bench.py per-layer timings (CB_ARGS, default --fp32) with the in-tree
#                    library and with the variant build DIR/_hcb_kernels.so (tools/build_variant.py)
#   prof[:args]      rocprofv3 --kernel-trace --stats of bench.py, summarised by tools/kstats.py
#   pmc:COUNTERS     one rocprofv3 --pmc pass (counters comma-separated) over bench.py --steps 3
#   dpsweep[:dtype]  forced 1-rank DP path (native RCCL engine): backward_segments stage|block x
#                    HOROVOD_FUSION_THRESHOLD 32/64/128 MiB, against the single-graph step
#   readme           tools/gpu_readme_numbers.sh
#   race             tools/race_full.py (serialised vs async bitwise race check at full size)
#   py:SCRIPT[,args] python SCRIPT args (a probe / diagnostic)
# env: TAG (output prefix), PYTEST_X (default -x; PYTEST_X= runs every test), PYTEST_K (-k filter),
#      BENCH_ARGS (extra bench.py arguments of benchab, e.g. "--model inception3 --secondary none")
# Outputs go to gpurun_out/${TAG}_<step>.*
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG

fail() { echo "FAILED: $1"; [ -f "$2" ] && tail -40 "$2"; exit 1; }

for step in "$@"; do
  name=${step%%:*}; arg=""; [ "$name" != "$step" ] && arg=${step#*:}
  args=${arg//,/ }
  case $name in
    smoke)
      timeout -k 10 300 python __graft_entry__.py smoke > ${O}_smoke.log 2>&1 || fail smoke ${O}_smoke.log
      tail -1 ${O}_smoke.log ;;
    tests)
      files=${args:-tests}
      timeout -k 10 900 python -u -m pytest $files ${PYTEST_K:+-k "$PYTEST_K"} -m gpu ${PYTEST_X--x} -v -s \
        --timeout 300 --timeout-method thread \
        > ${O}_tests.log 2>&1 || fail tests ${O}_tests.log
      tail -1 ${O}_tests.log ;;
    bench)
      timeout -k 10 400 python bench.py $args > ${O}_bench.json 2> ${O}_bench.err || fail bench ${O}_bench.err
      cut -c1-260 ${O}_bench.json ;;
    benchab)  # ABBA: base var var base (a drift between consecutive runs cancels)
      for r in 1 2; do if [ $r = 1 ]; then vs="base var"; else vs="var base"; fi; for v in $vs; do
        if [ $v = base ]; then e=""; else e="$args"; fi
        env $e timeout -k 10 400 python bench.py --steps 40 --warmup 10 $BENCH_ARGS > ${O}_ab.json 2> ${O}_ab.err || fail benchab ${O}_ab.err
        echo "$v [$e] $(python -c "import json;d=json.load(open('${O}_ab.json'));print(d['value'], d['ms_per_step'], 'bf16', d.get('bf16_value'), d.get('bf16_ms_per_step'))")"
      done; done ;;
    convab)
      for v in base var; do
        if [ $v = base ]; then e=""; else e="HCB_KERNELS_SO=$args/_hcb_kernels.so"; fi
        env $e timeout -k 10 300 python tools/conv_bench.py ${CB_ARGS:---fp32} > ${O}_conv_$v.txt 2>&1 \
          || fail convab ${O}_conv_$v.txt
        echo "$v [$e] $(tail -1 ${O}_conv_$v.txt)"
      done ;;
    prof)
      pargs=${args:---steps 10 --warmup 3}
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d ${O}_prof -o run \
        -- python $R/bench.py $pargs > ${O}_prof.log 2>&1) || fail prof ${O}_prof.log
      steps=$(python -c "import sys;a=sys.argv[1:];s=int(a[a.index('--steps')+1]) if '--steps' in a else 10;w=int(a[a.index('--warmup')+1]) if '--warmup' in a else 3;print(s+w)" $pargs)
      python tools/kstats.py ${O}_prof/run_kernel_stats.csv --steps $steps > ${O}_kstats.txt || fail kstats
      sed -n '/per class/,$p' ${O}_kstats.txt ;;
    pmc)
      (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $args --kernel-trace --output-format csv -d ${O}_pmc -o run \
        -- python $R/bench.py --steps 3 --warmup 2 > ${O}_pmc.log 2>&1) || fail pmc ${O}_pmc.log
      echo "pmc done: ${O}_pmc" ;;
    dpsweep)
      dt=${args:-fp32}
      common="--compute_dtype $dt --secondary none --steps 40 --warmup 10"
      timeout -k 10 400 python bench.py $common > ${O}_dp.json 2> ${O}_dp.err || fail dpsweep ${O}_dp.err
      echo "single-graph $(python tools/jfield.py ${O}_dp.json value ms_per_step)" | tee ${O}_dpsweep.txt
      for seg in stage block; do for mb in 32 64 128; do
        HOROVOD_FUSION_THRESHOLD=$((mb << 20)) timeout -k 10 400 python bench.py $common --force_dp_path \
          --backward_segments $seg > ${O}_dp.json 2> ${O}_dp.err || fail dpsweep ${O}_dp.err
        echo "dp seg=$seg bucket=${mb}MiB $(python tools/jfield.py ${O}_dp.json value ms_per_step comm)" \
          | tee -a ${O}_dpsweep.txt
      done; done ;;
    readme)
      bash tools/gpu_readme_numbers.sh || fail readme ;;
    race)
      timeout -k 10 1000 python -u tools/race_full.py $args > ${O}_race.txt 2>&1 || fail race ${O}_race.txt
      tail -5 ${O}_race.txt ;;
    py)
      timeout -k 10 600 python -u $args > ${O}_py.log 2>&1 || fail py ${O}_py.log
      tail -40 ${O}_py.log ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
done
echo "gpu_run done: $*"
