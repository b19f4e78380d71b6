#!/usr/bin/env python3
"""Time every forward tile config (generic implicit GEMM cfg 0-16 and the LDS-resident-patch
3x3 kernels cfg 17-21, with their split-K factors) on the ResNet-50 3x3 / stride-1 layers, and
print them sorted, with each config's modelled L2 -> LDS bytes per step (the quantity the patch
kernels cut: the generic kernel fetches the im2col A tile once per filter tap).

    python tools/patch_sweep.py [--batch 64] [--reps 20] [--pass fwd|dgrad]
"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.nn.layers import ConvBN
from azure_hc_intel_tf_amd.ops import functional as Fn


def fetched_mb(cfg, M, N, C, H, W):
    """modelled bytes moved L2 -> LDS by all blocks of one launch (MB)"""
    bm, bn = Fn._CONV_TILES[cfg]
    tiles_m, tiles_n = math.ceil(M / bm), math.ceil(N / bn)
    K = 9 * C
    b = tiles_m * tiles_n * K * bn * 2  # weight tiles
    if cfg in Fn.PATCH_CFGS:
        span = bm + 2 * math.ceil(bm / W) + 2 * (W + 2) + 3  # typical (non image-crossing) patch
        b += tiles_m * tiles_n * (C // 64) * span * 128
    else:
        b += tiles_m * tiles_n * K * bm * 2
    return b / 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--pass", dest="which", default="fwd", choices=["fwd", "dgrad"])
    ap.add_argument("--cfgs", default=None, help="comma-separated cfg ids (default: every candidate)")
    ap.add_argument("--stages", default=None, help="comma-separated stage numbers, e.g. 3,4")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    only_cfgs = None if a.cfgs is None else {int(c) for c in a.cfgs.split(",")}
    only_stages = None if a.stages is None else {f"stage{s}/" for s in a.stages.split(",")}
    dev = torch.device("cuda")
    m = create_model("resnet50", device=dev, compute_dtype="bf16" if str(dev).startswith("cuda") else None)
    m.ps.repack()
    seen = set()
    for layer in m.all_layers():
        if not isinstance(layer, ConvBN) or not Fn.patch_eligible(layer.spec):
            continue
        s = layer.spec
        H, W, C = layer.in_shape
        P, Q, K = layer.out_shape
        if (H, C, K) in seen or (only_stages and not any(layer.name.startswith(t) for t in only_stages)):
            continue
        seen.add((H, C, K))
        N = a.batch
        M = N * P * Q
        x = torch.randn(N, H, W, C, device=dev).bfloat16()
        dz = torch.randn(N, P, Q, K, device=dev).bfloat16()
        y = torch.empty(N, P, Q, K, device=dev, dtype=torch.bfloat16)
        dx = torch.zeros(N, H, W, C, device=dev, dtype=torch.bfloat16)
        acc = torch.zeros(8 * 2 * max(C, K), device=dev)
        ncol = K if a.which == "fwd" else C
        rows = []
        for cfg in Fn.fwd_candidates(ncol, True):
            if only_cfgs is not None and cfg not in only_cfgs:
                continue
            for sp in Fn.splitk_candidates(cfg, M, ncol, 9 * (C if a.which == "fwd" else K)):
                plan = cfg if sp == 1 else [cfg, sp]
                if a.which == "fwd":
                    fn = lambda: Fn.conv_forward(x, s, layer.pack.pack, None, y, stats=acc, stats_R=8, cfg=plan)
                else:
                    fn = lambda: Fn.conv_dgrad(dz, s, layer.pack.tr, None, dx, False, cfg=plan)
                for _ in range(3):
                    fn()
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(a.reps):
                    fn()
                en.record()
                en.synchronize()
                us = st.elapsed_time(en) / a.reps * 1000
                cin = C if a.which == "fwd" else K
                rows.append((us, cfg, sp, fetched_mb(cfg, M, ncol, cin, W, W)))
        rows.sort()
        flop = 2.0 * M * ncol * 9 * (C if a.which == "fwd" else K)
        print(f"== {layer.name} {a.which} M={M} N={ncol} K={9 * (C if a.which == 'fwd' else K)} H={H}", flush=True)
        for us, cfg, sp, mb in rows[:a.top]:
            tag = "patch" if cfg in Fn.PATCH_CFGS else ("igemm-ku2" if cfg >= 22 else "igemm")
            print(f"   cfg {cfg:2d} x{sp} {tag} {Fn._CONV_TILES[cfg]}: {us:7.1f} us  {flop / us / 1e6:6.0f} TF  "
                  f"fetch {mb:6.0f} MB = {mb / us:5.1f} TB/s", flush=True)


if __name__ == "__main__":
    main()
