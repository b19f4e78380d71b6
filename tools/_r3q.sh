timeout -k 10 300 python -u tools/diag_fp32_shallow.py --bn > gpurun_out/r3q.txt 2>&1
timeout -k 10 300 python -u tools/diag_fp32_shallow.py --bn --bf16-first >> gpurun_out/r3q.txt 2>&1
