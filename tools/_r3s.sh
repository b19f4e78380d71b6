timeout -k 10 300 python -u tools/diag_fp32_shallow.py --both > gpurun_out/r3s.txt 2>&1
timeout -k 10 300 python -u tools/diag_fp32_shallow.py --both --bf16-first >> gpurun_out/r3s.txt 2>&1
