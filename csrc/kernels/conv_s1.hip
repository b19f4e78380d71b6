// Forward / data-gradient GEMM of the 16-bit builds (bf16, or IEEE fp16 in _hcb_kernels_f16.so) on
// the fp32 path's plane-GEMM kernel (conv_p3_fwd.h) with ONE operand plane: 32- or 64-deep slots,
// early-release LDS-DMA rings, register-pipelined fragments, tiles sized for one to three
// workgroups per CU, the 16-bit epilogue (BN statistics, fused BN backward, beta-accumulate).
// Offered to the autotuner beside conv_igemm.hip's configs as cfg CONV_S1_BASE + i of the
// conv_igemm op (i = the plane-GEMM cfg index, conv_p3_fwd.h).
#include "conv_p3_fwd.h"

namespace hcb {

void launch_conv_s1(const ConvParams& p, int cfg, hipStream_t st) {
  if (p.bnb_acc != nullptr)
    launch_p3_cfg<true, false, 1>(p, cfg, st);
  else
    launch_p3_cfg<false, false, 1>(p, cfg, st);
}

}  // namespace hcb
