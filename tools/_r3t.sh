timeout -k 10 300 python -u tools/diag_fp32_shallow.py --saved > gpurun_out/r3t.txt 2>&1
timeout -k 10 300 python -u tools/diag_fp32_shallow.py --saved --bf16-first >> gpurun_out/r3t.txt 2>&1
