timeout -k 10 300 python -u tools/diag_fp32_shallow.py --scan > gpurun_out/r3o_scan.txt 2>&1
