#!/usr/bin/env python3
"""A/B of the weight-gradient loaders in ONE process: every distinct ResNet-50 conv layer at its
autotuned (cfg, splits), original divide-per-row loaders (set_wgrad_ri(0)) vs the
row-incremental ones with per-lane rows (2) and shared rows (1, default), interleaved rounds,
median us.

    python tools/wgrad_ab.py [--batch 64] [--model resnet50]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.nn.layers import ConvBN
from azure_hc_intel_tf_amd.ops import _ext, autotune
from azure_hc_intel_tf_amd.ops import functional as Fn


def tm(fn, reps=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--model", default="resnet50")
    a = ap.parse_args()
    dev = torch.device("cuda")
    hcb = _ext.ops()
    autotune.load_cache()
    m = create_model(a.model, device=dev)
    seen = {}
    for l in m.all_layers():
        if not isinstance(l, ConvBN) or l.name == "conv0":
            continue
        s = l.spec
        N = a.batch
        H, W, C = l.in_shape
        P, Q, K = l.out_shape
        key = (H, W, C, P, Q, K, s.kh, s.sh)
        if key in seen:
            seen[key][1] += 1
            continue
        seen[key] = [l.name, 1, N, l]
    tot = [0.0, 0.0, 0.0]
    print(f"{'layer':28s} {'cfg':>8s}  orig us  RI-lane  RI-shared  speedup  TF")
    for key, (name, cnt, N, l) in seen.items():
        s = l.spec
        H, W, C = l.in_shape
        P, Q, K = l.out_shape
        x = torch.randn(N, H, W, C, device=dev).bfloat16()
        dz = torch.randn(N, P, Q, K, device=dev).bfloat16()
        dw = torch.zeros(K, s.K, device=dev)
        M = N * P * Q
        cfg = Fn.wgrad_cfg(K, s.K, M, s.kh * s.kw)
        ts = {0: [], 1: [], 2: []}
        for _ in range(5):
            for ri in (0, 2, 1):
                hcb.set_wgrad_ri(ri)
                ts[ri].append(tm(lambda: Fn.conv_wgrad(dz, x, s, dw, cfg=tuple(cfg))))
        hcb.set_wgrad_ri(1)
        t0, t1, t2 = statistics.median(ts[0]), statistics.median(ts[1]), statistics.median(ts[2])
        tot[0] += cnt * t0
        tot[1] += cnt * t1
        tot[2] += cnt * t2
        fl = 2.0 * M * K * s.K
        print(f"{name:28s} {str(tuple(cfg)):>8s} {t0:7.1f} {t2:7.1f} {t1:7.1f}  {t0 / t1:5.2f}x  {fl / t1 / 1e6:5.0f}  x{cnt}",
              flush=True)
    print(f"TOTAL per step (us): orig {tot[0]:.1f}  RI per-lane {tot[2]:.1f}  RI shared {tot[1]:.1f}")


if __name__ == "__main__":
    main()
