#!/usr/bin/env python3
"""Time every weight-gradient (cfg, split-K) candidate on the ResNet-50 layers and print the
best time per tile config and layer (which kernel family wins where).

    python tools/wgrad_sweep.py [--batch 64] [--layers stage3/block2/conv2,...]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.nn.layers import ConvBN
from azure_hc_intel_tf_amd.ops import functional as Fn
from azure_hc_intel_tf_amd.ops.autotune import _time


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--layers", default="")
    a = ap.parse_args()
    dev = torch.device("cuda")
    m = create_model("resnet50", device=dev, compute_dtype="bf16" if str(dev).startswith("cuda") else None)
    seen = set()
    want = set(a.layers.split(",")) if a.layers else None
    for l in m.all_layers():
        if not isinstance(l, ConvBN):
            continue
        if want and l.name not in want:
            continue
        s = l.spec
        H, W, C = l.in_shape
        P, Q, K = l.out_shape
        key = (H, W, C, P, Q, K, s.kh, s.sh)
        if key in seen:
            continue
        seen.add(key)
        N = a.batch
        M = N * P * Q
        x = torch.randn(N, H, W, C, device=dev).bfloat16()
        dz = torch.randn(N, P, Q, K, device=dev).bfloat16()
        dw = torch.zeros(K, s.K, device=dev)
        best = {}
        for cfg, sp in Fn.wgrad_candidates(K, s.K, M):
            t = _time(lambda: Fn.conv_wgrad(dz, x, s, dw, cfg=(cfg, sp)), reps=10) * 1000
            if cfg not in best or t < best[cfg][0]:
                best[cfg] = (t, sp)
        flops = 2.0 * M * K * s.K
        row = " ".join(f"c{c}:{t:6.1f}/{sp:<3d}" for c, (t, sp) in sorted(best.items()))
        bc = min(best, key=lambda c: best[c][0])
        print(f"{l.name:26s} {K:5d}x{s.K:5d} M={M:7d} best c{bc} {best[bc][0]:6.1f}us "
              f"{flops / best[bc][0] / 1e6:6.0f}TF | {row}", flush=True)


if __name__ == "__main__":
    main()
