#!/usr/bin/env python3
"""Per-layer ceiling check: each ResNet-50 conv GEMM (fwd and weight-grad) against hipBLASLt
(torch.matmul, bf16) on a dense GEMM of the same M x N x K -- no im2col, no fused BN
statistics, so hipBLASLt's time is an optimistic bound on what a library GEMM gets on the
shape. Tells whether a layer's gap to the MFMA peak is the shape (small M, N or K) or our
kernel.

    python tools/gemm_equiv.py [--batch 64]
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    dev = torch.device("cuda")
    m = create_model("resnet50", device=dev, compute_dtype="bf16" if str(dev).startswith("cuda") else None)
    m.ps.repack()
    autotune.load_cache()
    seen = set()
    tot = {"fwd": 0.0, "blas_fwd": 0.0, "wgrad": 0.0, "blas_wgrad": 0.0}
    print(f"{'layer':28s} {'M':>7s} {'N':>5s} {'K':>5s} | fwd us (TF)   blasLt us (TF) | wgrad us (TF) blasLt us (TF)")
    for l in m.all_layers():
        if not isinstance(l, ConvBN) or l.name == "conv0":
            continue
        s = l.spec
        N = a.batch
        H, W, C = l.in_shape
        P, Q, K = l.out_shape
        M, Kg = N * P * Q, s.K
        key = (M, K, Kg, s.kh)
        cnt = 1
        if key in seen:
            continue
        seen.add(key)
        cnt = sum(1 for q in m.all_layers() if isinstance(q, ConvBN) and q.name != "conv0"
                  and (N * q.out_shape[0] * q.out_shape[1], q.out_shape[2], q.spec.K, q.spec.kh) == key)
        x = torch.randn(N, H, W, C, device=dev).bfloat16()
        dz = torch.randn(N, P, Q, K, device=dev).bfloat16()
        y = torch.empty(N, P, Q, K, device=dev, dtype=torch.bfloat16)
        acc = torch.zeros(8 * 2 * K, device=dev)
        dw = torch.zeros(K, Kg, device=dev)
        t_f = tm(lambda: Fn.conv_forward(x, s, l.pack.pack, None, y, stats=acc, stats_R=8))
        t_w = tm(lambda: Fn.conv_wgrad(dz, x, s, dw))
        A = torch.randn(M, Kg, device=dev).bfloat16()
        B = torch.randn(Kg, K, device=dev).bfloat16()
        C2 = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        t_bf = tm(lambda: torch.matmul(A, B, out=C2))
        dz2 = dz.view(M, K)
        Xw = torch.randn(M, Kg, device=dev).bfloat16()
        W2 = torch.empty(K, Kg, device=dev, dtype=torch.bfloat16)
        t_bw = tm(lambda: torch.matmul(dz2.t(), Xw, out=W2))
        fl = 2.0 * M * K * Kg
        tf = lambda t: fl / (t * 1e-6) / 1e12
        print(f"{l.name:28s} {M:7d} {K:5d} {Kg:5d} | {t_f:7.1f} ({tf(t_f):4.0f}) {t_bf:7.1f} ({tf(t_bf):4.0f})  | "
              f"{t_w:7.1f} ({tf(t_w):4.0f}) {t_bw:7.1f} ({tf(t_bw):4.0f})  x{cnt}")
        tot["fwd"] += cnt * t_f
        tot["blas_fwd"] += cnt * t_bf
        tot["wgrad"] += cnt * t_w
        tot["blas_wgrad"] += cnt * t_bw
    print("TOTAL per step (us, counts applied):", {k: round(v, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
