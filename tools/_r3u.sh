timeout -k 10 300 python -u tools/diag_fp32_shallow.py --gap > gpurun_out/r3u.txt 2>&1
timeout -k 10 300 python -u tools/diag_fp32_shallow.py --gap --bf16-first >> gpurun_out/r3u.txt 2>&1
