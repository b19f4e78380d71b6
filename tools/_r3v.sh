timeout -k 10 300 python -u tools/diag_fp32_shallow.py --bncmp > gpurun_out/r3v.txt 2>&1
timeout -k 10 300 python -u tools/diag_fp32_shallow.py --bncmp --bf16-first >> gpurun_out/r3v.txt 2>&1
