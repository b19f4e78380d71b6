#!/usr/bin/env python3
"""Time the ResNet-50 stem conv (fwd + wgrad, bs=64, 224x224) in its direct padded 7x7/2 form
and in the space-to-depth 4x4/1 form (nn/layers.StemS2D), every kernel config of each."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from azure_hc_intel_tf_amd.nn.layers import ConvBN, StemS2D
from azure_hc_intel_tf_amd.nn.params import ParamStore
from azure_hc_intel_tf_amd.ops import autotune
from azure_hc_intel_tf_amd.ops import functional as Fn


def t_us(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1000


def main():
    autotune.load_cache()
    dev = torch.device("cuda")
    N = 64
    ps = ParamStore(seed=1)
    d = ConvBN(ps, "direct", (224, 224, 8), 64, 7, 7, 2, 2, "SAME_RESNET", need_dx=False, logical_cin=3)
    f = StemS2D(ps, "fold", (224, 224, 8), 64, need_dx=False, logical_cin=3)
    ps.finalize(dev)
    ps.repack()
    x = torch.randn(N, 224, 224, 8, device=dev).bfloat16()
    z = torch.empty(N, 112, 112, 64, device=dev, dtype=torch.bfloat16)
    dz = torch.randn(N, 112, 112, 64, device=dev).bfloat16()
    acc = torch.zeros(8 * 2 * 64, device=dev)
    xf = f.fold_input(x)
    wf = f._folded_weight(dev)
    dw = torch.zeros(64, d.spec.K, device=dev)
    dwf = torch.zeros(64, 256, device=dev)
    print(f"fold input: {t_us(lambda: f.fold_input(x)):.1f} us   fold weight: {t_us(lambda: f._folded_weight(dev)):.1f} us")
    for name, spec, inp, w, dws in (("direct", d.spec, x, d.pack.pack, dw), ("s2d", f.fold_spec, xf, wf, dwf)):
        M = N * 112 * 112
        best = min((t_us(lambda: Fn.conv_forward(inp, spec, w, None, z, stats=acc, stats_R=8, cfg=c)), c)
                   for c in Fn.fwd_candidates(64))
        tuned = t_us(lambda: Fn.conv_forward(inp, spec, w, None, z, stats=acc, stats_R=8))
        wb = min((t_us(lambda: Fn.conv_wgrad(dz, inp, spec, dws, cfg=(c, s_))), (c, s_))
                 for c, s_ in Fn.wgrad_candidates(64, spec.K, M))
        wt = t_us(lambda: Fn.conv_wgrad(dz, inp, spec, dws))
        print(f"{name:7s} K={spec.K:4d} fwd tuned {tuned:7.1f} us (best {best[0]:7.1f} cfg {best[1]})   "
              f"wgrad tuned {wt:7.1f} us (best {wb[0]:7.1f} cfg {wb[1]})")


if __name__ == "__main__":
    main()
