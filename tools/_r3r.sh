timeout -k 10 300 python -u tools/diag_fp32_shallow.py --ref > gpurun_out/r3r.txt 2>&1
timeout -k 10 300 python -u tools/diag_fp32_shallow.py --ref --bf16-first >> gpurun_out/r3r.txt 2>&1
