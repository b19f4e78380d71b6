// Weight gradient of the 16-bit builds (bf16, or IEEE fp16 in _hcb_kernels_f16.so) on the fp32
// path's slot-ring kernel (conv_p3_wgrad.h) with ONE operand plane: 32- or 64-deep pixel-row
// slots, early-release rings, register-pipelined transposed fragment reads, tiles sized for one to
// four workgroups per CU. Offered to the autotuner beside conv_wgrad.hip's kernels as cfg
// WGRAD_S1_BASE + i of the conv_wgrad op.
#include "conv_p3_wgrad.h"

namespace hcb {

// s1 cfg (block tile, waves x wave tile, slots x pixel rows, workgroups per CU):
//   0 128x128 (2x2 of 64x64, 3x32, 2)   1 128x128 (2x2 of 64x64, 2x64, 2)   2 128x128 (2x4 of 64x32, 3x32, 2)
//   3 256x128 (4x2 of 64x64, 2x32, 1)   4 128x64 (2x2 of 64x32, 3x32, 3)    5 64x64 (2x2 of 32x32, 3x32, 4)
//   6 64x128 (2x2 of 32x64, 3x32, 3)    7 128x128 (2x2 of 64x64, 3x64, 1)
void launch_wgrad_s1(const WgradParams& p, int cfg, int splits, hipStream_t st) {
  switch (cfg) {
    case 0: wlaunch_p3<2, 2, 64, 64, 3, 32, 2, 1>(p, splits, st); break;
    case 1: wlaunch_p3<2, 2, 64, 64, 2, 64, 2, 1>(p, splits, st); break;
    case 2: wlaunch_p3<2, 4, 64, 32, 3, 32, 2, 1>(p, splits, st); break;
    case 3: wlaunch_p3<4, 2, 64, 64, 2, 32, 1, 1>(p, splits, st); break;
    case 4: wlaunch_p3<2, 2, 64, 32, 3, 32, 3, 1>(p, splits, st); break;
    case 5: wlaunch_p3<2, 2, 32, 32, 3, 32, 4, 1>(p, splits, st); break;
    case 6: wlaunch_p3<2, 2, 32, 64, 3, 32, 3, 1>(p, splits, st); break;
    default: wlaunch_p3<2, 2, 64, 64, 3, 64, 1, 1>(p, splits, st); break;
  }
}

}  // namespace hcb
