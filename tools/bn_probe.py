#!/usr/bin/env python3
"""Streaming efficiency of the BN apply kernels (forward apply, forward apply + residual, backward
apply of a pre-reduced gradient) on the ResNet-50 bs64 tensor shapes, against torch elementwise
kernels that move the same bytes (copy 1R1W, add 2R1W)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from azure_hc_intel_tf_amd.ops import functional as Fn


def tm(fn, reps=30):
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
    dev = "cuda"
    R = 8
    print(f"{'M x C':>14s} {'MB':>6s} | fwd us  TB/s | fwd+res  TB/s | bwd  TB/s | torch copy TB/s  add TB/s")
    for M, C in [(200704, 64), (200704, 256), (50176, 128), (50176, 512), (12544, 256), (12544, 1024), (3136, 512),
                 (3136, 2048)]:
        z = torch.randn(M, C, device=dev).bfloat16().view(M, 1, 1, C)
        y = torch.empty_like(z)
        r = torch.randn_like(z)
        g = torch.randn_like(z)
        gamma, beta = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        acc = torch.rand(R * 2 * C, device=dev) * M / R
        sm, si = torch.empty(C, device=dev), torch.empty(C, device=dev)
        dg, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
        mb = M * C * 2 / 1e6
        t_f = tm(lambda: Fn.bn_forward_acc(z, gamma, beta, rm, rv, 0.9, 1e-5, y, True, acc, R, sm, si))
        t_r = tm(lambda: Fn.bn_forward_acc(z, gamma, beta, rm, rv, 0.9, 1e-5, y, True, acc, R, sm, si, residual=r))
        saved = Fn.BNSaved(sm, si)
        t_b = tm(lambda: Fn.bn_backward_acc(g, None, z, saved, gamma, beta, 0, dg, db, y, acc, R, pre_reduced=True))
        t_c = tm(lambda: y.copy_(z))
        t_a = tm(lambda: torch.add(z, r, out=y))
        bw = lambda n, t: n * mb / t  # MB/us = TB/s
        print(f"{M:7d} x {C:4d} {mb:6.1f} | {t_f:6.1f} {bw(2, t_f):4.2f} | {t_r:6.1f} {bw(3, t_r):4.2f} | {t_b:6.1f} "
              f"{bw(3, t_b):4.2f} | {t_c:6.1f} {bw(2, t_c):4.2f} {t_a:6.1f} {bw(3, t_a):4.2f}", flush=True)


if __name__ == "__main__":
    main()
