timeout -k 10 300 python -u tools/wgrad_split_sweep.py > gpurun_out/y_split.txt 2>&1; rc=$?; cat gpurun_out/y_split.txt; exit $rc
