#!/usr/bin/env python3
"""Run ONE conv GEMM of a model layer repeatedly (a target for rocprofv3 --pmc passes / traces):

    python tools/layer_probe.py --layer stage3/block1/conv2 --op fwd [--fp32] [--cfg 7,1] [--reps 50]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.nn.layers import ConvBN
from azure_hc_intel_tf_amd.ops import autotune
from azure_hc_intel_tf_amd.ops import functional as Fn


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--layer", default="stage3/block1/conv2")
    ap.add_argument("--op", default="fwd", choices=["fwd", "dgrad", "wgrad"])
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--fp32", action="store_true")
    ap.add_argument("--cfg", default=None, help="cfg[,splits] (default: tuned)")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--stats_r", type=int, default=8,
                    help="fwd: BN-statistics replicas of the epilogue (-1: no statistics, 0: per-tile slab)")
    ap.add_argument("--bnb", type=int, default=-1,
                    help="dgrad: fuse the consuming BN's backward reduction (ReLU mode 0/1/2) into the epilogue")
    a = ap.parse_args()
    dev = torch.device("cuda")
    m = create_model(a.model, device=dev, compute_dtype="fp32" if a.fp32 else None)
    m.ps.repack()
    autotune.load_cache()
    l = [x for x in m.all_layers() if isinstance(x, ConvBN) and x.name == a.layer][0]
    s = l.spec
    N = a.batch
    H, W, C = l.in_shape
    P, Q, K = l.out_shape
    mk = (lambda sh: Fn.to_planes(torch.randn(sh, device=dev))) if a.fp32 else (
        lambda sh: torch.randn(sh, device=dev).bfloat16())
    odt = torch.float32 if a.fp32 else torch.bfloat16
    cfg = None
    if a.cfg:
        v = [int(t) for t in a.cfg.split(",")]
        cfg = (v[0], v[1] if len(v) > 1 else 1)
    if a.op == "fwd":
        x, y = mk((N, H, W, C)), torch.empty(N, P, Q, K, device=dev, dtype=odt)
        R = a.stats_r
        acc = torch.zeros(max(R, 1) * 2 * K if R != 0 else (N * P * Q // 16 + 1) * 2 * K, device=dev)
        fn = lambda: Fn.conv_forward(x, s, l.pack.pack, None, y, stats=acc if R >= 0 else None, stats_R=max(R, 0),
                                     cfg=cfg)
    elif a.op == "dgrad":
        dz, dx = mk((N, P, Q, K)), torch.zeros(N, H, W, C, device=dev, dtype=odt)
        bnb = None
        if a.bnb >= 0:
            z = torch.randn(N, H, W, C, device=dev)
            yb = Fn.to_planes(torch.relu(z)) if a.fp32 else torch.relu(z).bfloat16()
            st = Fn.BNSaved(torch.zeros(C, device=dev), torch.ones(C, device=dev))
            bacc = torch.zeros(8, 2, C, device=dev)
            bnb = Fn.BNBwdFuse(z if a.fp32 else z.bfloat16(), yb, st, torch.ones(C, device=dev),
                               torch.zeros(C, device=dev), a.bnb, bacc, 8)
        fn = lambda: Fn.conv_dgrad(dz, s, l.pack.tr, None, dx, False, cfg=cfg, bnb=bnb)
    else:
        x, dz = mk((N, H, W, C)), mk((N, P, Q, K))
        dw = torch.zeros(K, s.K, device=dev)
        fn = lambda: Fn.conv_wgrad(dz, x, s, dw, cfg=cfg)
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        fn()
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) / a.reps * 1000
    fl = 2.0 * N * P * Q * K * s.kh * s.kw * s.cin
    print(f"{a.layer} {a.op} cfg={cfg} {us:.1f} us  {fl / us / 1e6:.0f} TF (x6 MFMA: {6 * fl / us / 1e6 / 25:.0f}% of 2.5 PF)"
          if a.fp32 else f"{a.layer} {a.op} cfg={cfg} {us:.1f} us  {fl / us / 1e6:.0f} TF")


if __name__ == "__main__":
    main()
