#!/usr/bin/env python3
"""Run ONE ResNet-50 conv problem (fwd / dgrad / wgrad) with a fixed kernel config many times:
the target for rocprofv3 counter collection of a single kernel.

    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES ... -- python tools/conv_micro.py \
        --layer stage3/block1/conv2 --pass fwd --cfg 4 --reps 20
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.nn.layers import ConvBN
from azure_hc_intel_tf_amd.ops import functional as Fn


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--layer", default="stage3/block1/conv2")
    ap.add_argument("--pass", dest="which", default="fwd", choices=["fwd", "dgrad", "wgrad"])
    ap.add_argument("--cfg", type=int, default=None)
    ap.add_argument("--splits", type=int, default=None)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    from azure_hc_intel_tf_amd.ops import autotune

    autotune.load_cache()  # --cfg omitted: the autotuned config of this shape
    m = create_model(a.model, device=dev, compute_dtype="bf16" if str(dev).startswith("cuda") else None)
    m.ps.repack()
    layer = next(l for l in m.all_layers() if isinstance(l, ConvBN) and l.name == a.layer)
    s = layer.spec
    N = a.batch
    H, W, C = layer.in_shape
    P, Q, K = layer.out_shape
    x = torch.randn(N, H, W, C, device=dev).bfloat16()
    dz = torch.randn(N, P, Q, K, device=dev).bfloat16()
    if a.which == "fwd":
        y = torch.empty(N, P, Q, K, device=dev, dtype=torch.bfloat16)
        acc = torch.zeros(8 * 2 * K, device=dev)
        fn = lambda: Fn.conv_forward(x, s, layer.pack.pack, None, y, stats=acc, stats_R=8, cfg=a.cfg)
    elif a.which == "dgrad":
        dx = torch.zeros(N, H, W, C, device=dev, dtype=torch.bfloat16)
        fn = lambda: Fn.conv_dgrad(dz, s, layer.pack.tr, None, dx, False, cfg=a.cfg)
    else:
        dw = torch.zeros(K, s.K, device=dev)
        cfg = None if a.cfg is None else (a.cfg, a.splits or 1)
        fn = lambda: Fn.conv_wgrad(dz, x, s, dw, cfg=cfg)
    for _ in range(a.reps):
        fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(a.reps):
        fn()
    en.record()
    en.synchronize()
    us = st.elapsed_time(en) / a.reps * 1000
    fl = 2.0 * N * P * Q * K * s.kh * s.kw * s.cin
    print(f"{a.layer} {a.which} cfg={a.cfg}: {us:.1f} us  {fl / us / 1e6:.0f} TF/s")


if __name__ == "__main__":
    main()
