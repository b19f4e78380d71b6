#!/usr/bin/env python3
"""Split-K sweep of the weight-gradient GEMM of the ResNet-50 3x3 layers (bs64) at a fixed tile
config: time per split count next to the fp32 atomic bytes it adds (splits x |dW| x 4 B), to see
how much of the kernel the memory-side atomics account for (~1.3 TB/s chip-wide)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.nn.layers import ConvBN
from azure_hc_intel_tf_amd.ops import autotune
from azure_hc_intel_tf_amd.ops import functional as Fn


def tm(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1000.0


def main():
    dev = torch.device("cuda")
    autotune.load_cache()
    m = create_model("resnet50", device=dev, compute_dtype="bf16" if str(dev).startswith("cuda") else None)
    N = 64
    done = set()
    for l in m.all_layers():
        if not isinstance(l, ConvBN) or l.spec.kh != 3 or l.name in done:
            continue
        key = (l.in_shape, l.out_shape)
        if key in done:
            continue
        done.add(key)
        s = l.spec
        H, W, C = l.in_shape
        P, Q, K = l.out_shape
        x = torch.randn(N, H, W, C, device=dev).bfloat16()
        dz = torch.randn(N, P, Q, K, device=dev).bfloat16()
        dw = torch.zeros(K, s.K, device=dev)
        M = N * P * Q
        mb = K * s.K * 4 / 1e6
        print(f"{l.name}: dW {K}x{s.K} ({mb:.2f} MB), M={M}, tuned {Fn.wgrad_cfg(K, s.K, M, 9)}", flush=True)
        for cfg in (2, 13, 10):
            row = []
            for sp in (1, 2, 4, 8, 16, 32, 64, 128):
                if (M // 64) // sp < 2:
                    break
                t = tm(lambda: Fn.conv_wgrad(dz, x, s, dw, cfg=(cfg, sp)))
                row.append(f"s{sp}:{t:.1f}({sp * mb:.0f}MB)")
            print(f"  cfg {cfg:2d}: " + " ".join(row), flush=True)


if __name__ == "__main__":
    main()
