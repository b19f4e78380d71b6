timeout -k 10 300 python -u tools/diag_fp32_shallow.py --stages > gpurun_out/r3p.txt 2>&1
timeout -k 10 300 python -u tools/diag_fp32_shallow.py --stages --bf16-first >> gpurun_out/r3p.txt 2>&1
