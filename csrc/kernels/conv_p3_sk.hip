// Stream-K instantiations of the forward / data-gradient plane GEMM (conv_p3_fwd.h): every
// workgroup of a resident-sized grid reduces an even share of all (tile, k-slot) iterations, the
// shares of one tile meet through splitk_gather. Its own translation unit so it compiles in
// parallel with conv_p3.hip.
#include "conv_p3_fwd.h"

namespace hcb {

void launch_conv_p3_sk(const ConvParams& p, int cfg, hipStream_t st) {
  if (p.bnb_acc != nullptr)
    launch_p3_cfg<true, true>(p, cfg, st);
  else
    launch_p3_cfg<false, true>(p, cfg, st);
}

}  // namespace hcb
