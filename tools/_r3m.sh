set -o pipefail
mkdir -p gpurun_out
O=$PWD/gpurun_out/r3m_order.txt
: > $O
K=tests/test_determinism_gpu.py::test_shallow_net_gradients_elementwise_vs_fp32_cpu
run() {  # dir, pre-files
  (cd $1 && timeout -k 10 400 python -m pytest $2 $K -m gpu -q -s --timeout 300 > /tmp/r3m_run.log 2>&1)
  echo "dir=$1 pre=[$2] rc=$? $(grep -m1 'fp32 GPU grad check' /tmp/r3m_run.log | cut -c1-100) | $(tail -1 /tmp/r3m_run.log)" >> $O
}
run . ""
run . tests/test_comm_gpu.py
run abv/old tests/test_comm_gpu.py
run . tests/test_bn_shift_gpu.py
run . tests/test_data_gpu.py
