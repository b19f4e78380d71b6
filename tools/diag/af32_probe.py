#!/usr/bin/env python3
"""Prologue-side BN fusion prototype, per intra-block 1x1 edge of ResNet-50
(conv2's BN + ReLU consumed by conv3): the fused AF32 conv (fp32 z in, BN + ReLU + plane split in the
GEMM's A loader) against the unfused chain it would replace -- the BN apply pass (z -> planes,
bn_apply_acc, the production kernel) + the plane conv on every cfg the prototype has -- checked
against each other (same fp32 result to 3e-6) and timed in isolation (HIP events, --reps).

    python tools/diag/af32_probe.py [--batch 64] [--reps 50]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.nn.layers import ConvBN
from azure_hc_intel_tf_amd.ops import autotune
from azure_hc_intel_tf_amd.ops import functional as Fn


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda")
    m = create_model("resnet50", device=dev, compute_dtype="fp32")
    m.ps.repack()
    autotune.load_cache()
    layers = {x.name: x for x in m.all_layers() if isinstance(x, ConvBN)}
    N = a.batch
    tot_u = tot_f = 0.0
    for st, nb in ((1, 3), (2, 4), (3, 6), (4, 3)):
        name = f"stage{st}/block2/conv3"
        l = layers[name]
        s = l.spec
        H, W, C = l.in_shape
        P, Q, K = l.out_shape
        M = N * H * W
        torch.manual_seed(0)
        z = torch.randn(N, H, W, C, device=dev) * 2 + 0.3
        gamma, beta = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.2
        # the BN the apply pass derives from the statistics: feed it exact sums of z
        R = 8
        acc = torch.zeros(R, 2, C, device=dev)
        zz = z.view(-1, C).double()
        acc[0, 0] = zz.sum(0).float()
        acc[0, 1] = (zz * zz).sum(0).float()
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        smean, sinv = torch.empty(C, device=dev), torch.empty(C, device=dev)
        yp = Fn.Planes.empty((N, H, W, C), dev)
        apply = lambda: Fn.bn_forward_acc(z, gamma, beta, rm, rv, 0.0, 1e-5, yp, True, acc, R, smean, sinv)
        apply()
        torch.cuda.synchronize()
        sc = (gamma * sinv).contiguous()
        sh = (beta - smean * sc).contiguous()
        out_u = torch.empty(N, P, Q, K, device=dev)
        out_f = torch.empty(N, P, Q, K, device=dev)
        sacc = torch.zeros(R * 2 * K, device=dev)
        t_apply = timeit(apply, a.reps)
        best_u = best_f = None
        for cfg in (8, 13, 14, 15, 16, 18, 19, 20):
            conv_u = lambda: Fn.conv_forward(yp, s, l.pack.pack, None, out_u, stats=sacc, stats_R=R, cfg=(cfg, 1))
            tu = timeit(conv_u, a.reps)
            line = f"{name} M={M} C={C} K={K} cfg {cfg:2d}: unfused apply {t_apply:6.1f} + conv {tu:6.1f} = {t_apply + tu:6.1f} us"
            if best_u is None or tu < best_u[1]:
                best_u = (cfg, tu)
            conv_f = lambda: Fn.conv_forward_af32(z, s, l.pack.pack, out_f, sc, sh, cfg, stats=sacc, stats_R=R)
            if cfg <= 16 and conv_f():
                torch.cuda.synchronize()
                err = float((out_f - out_u).abs().max() / out_u.abs().max().clamp_min(1e-30))
                tf = timeit(conv_f, a.reps)
                line += f" | fused AF32 {tf:6.1f} us (max rel diff {err:.1e})"
                assert err < 3e-6, err
                if best_f is None or tf < best_f[1]:
                    best_f = (cfg, tf)
            print(line, flush=True)
        du, df = t_apply + best_u[1], best_f[1]
        tot_u += nb * du
        tot_f += nb * df
        print(f"{name}: best unfused {du:.1f} us (apply + cfg {best_u[0]}), best fused {df:.1f} us (cfg {best_f[0]}): "
              f"{du - df:+.1f} us per edge x {nb} blocks", flush=True)
    print(f"# all conv2->conv3 edges of the step (block2 shapes x blocks per stage): unfused {tot_u / 1000:.3f} ms, "
          f"fused {tot_f / 1000:.3f} ms ({(tot_u - tot_f) / 1000:+.3f} ms) -- before the plane write-out the "
          f"fused edge still owes the weight gradient (its x operand)")


if __name__ == "__main__":
    main()
