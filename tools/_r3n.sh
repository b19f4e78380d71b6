set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_fp32_shallow.py > gpurun_out/r3n_diag.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/diag_fp32_shallow.py --bf16-first >> gpurun_out/r3n_diag.txt 2>&1 || exit 1
