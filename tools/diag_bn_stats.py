#!/usr/bin/env python3
"""Repeat one ConvBN training forward and compare the conv-epilogue BN sums (acc_f, reduced over
its replicas) and the derived variance with an fp64 reference of the same bf16 GEMM."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from azure_hc_intel_tf_amd.nn.layers import ConvBN
from azure_hc_intel_tf_amd.nn.params import ParamStore
from azure_hc_intel_tf_amd.ops import functional as Fn

DEV = torch.device("cuda")


def main():
    ps = ParamStore(seed=3)
    layer = ConvBN(ps, "c", (28, 28, 64), 64, 1, 1, 1, 1, "SAME", relu=False, need_dx=False)
    ps.finalize(DEV)
    g = torch.Generator().manual_seed(7)
    layer.w.data.copy_((0.2 + 0.01 * torch.randn(layer.w.data.shape, generator=g)).to(DEV))
    ps.repack()
    x = (1.0 + torch.rand(64, 28, 28, 64, generator=torch.Generator().manual_seed(11))).bfloat16().to(DEV)
    w = layer.w.data.bfloat16().double().reshape(64, -1)
    z = x.double().reshape(-1, 64) @ w.t()
    M = z.shape[0]
    print("plan", Fn._plan(None, M, 64, layer.spec.K, DEV, 1), "K", layer.spec.K, "Kpad", layer.spec.Kpad)
    for shift in (False, True, True):
        K = layer.shift.data.double() if shift else torch.zeros(64, dtype=torch.float64, device=DEV)
        if not shift:
            layer.shift.data.zero_()
        r1 = (z - K).sum(0)
        r2 = ((z - K) ** 2).sum(0)
        rvar = z.var(0, unbiased=False)
        for it in range(3):
            ps.zero_stats()
            zz = layer.forward(x)
            torch.cuda.synchronize()
            acc = layer.acc_f.data.double().sum(0)
            var = layer.sv_invstd.data.double().pow(-2) - layer.eps
            e1 = ((acc[0] - r1).abs() / M / rvar.sqrt()).max().item()
            e2 = ((acc[1] - r2).abs() / (M * rvar)).max().item()
            ev = ((var - rvar).abs() / rvar)
            zerr = (layer._saved[1].double().reshape(-1, 64) - z).abs().max().item()
            print(f"shift={shift} it={it} S1err/std={e1:.2e} S2err/(M var)={e2:.2e} var_err={ev.max().item():.2e} "
                  f"at col {int(ev.argmax())} z_maxabs_err={zerr:.3f}", flush=True)
        layer.shift.data.copy_(layer.sv_mean.data)
    # the conv epilogue alone: atomics into R replicas vs the per-tile slab (plain stores)
    zb = torch.empty(64, 28, 28, 64, device=DEV, dtype=torch.bfloat16)
    rvar = z.var(0, unbiased=False)
    for K in (None, layer.shift.data):
        Kd = torch.zeros(64, dtype=torch.float64, device=DEV) if K is None else K.double()
        r2 = ((z - Kd) ** 2).sum(0)
        for R in (8, 1, 0):
            for cfg in (2, 0, 4):
                tiles = (M + 127) // 128 if cfg != 2 else (M + 63) // 64
                errs = []
                for it in range(4):
                    acc = torch.zeros((R if R else tiles) * 2 * 64, device=DEV)
                    Fn.conv_forward(x, layer.spec, layer.pack.pack, None, zb, stats=acc, stats_R=R, cfg=cfg,
                                    stats_shift=K)
                    torch.cuda.synchronize()
                    s2 = acc.view(-1, 2, 64).double().sum(0)[1]
                    errs.append(((s2 - r2).abs() / (M * rvar)).max().item())
                print(f"shift={K is not None} R={R} cfg={cfg}: S2 err " + " ".join(f"{e:.1e}" for e in errs), flush=True)


if __name__ == "__main__":
    main()
