#!/usr/bin/env python3
"""A/B of the LDS-DMA conv kernels' fragment schedule (hcb.set_igemm_variant) in ONE process,
interleaved rounds (guide rule 24): ResNet-50 bs64 conv problems at their tuned config
(forward and data-grad GEMMs) plus the big-GEMM probe, per variant: median over rounds."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.nn.layers import ConvBN
from azure_hc_intel_tf_amd.nn.params import ParamStore
from azure_hc_intel_tf_amd.ops import _ext, autotune
from azure_hc_intel_tf_amd.ops import functional as Fn


def t_us(fn, reps=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1000


def main():
    variants = [int(v) for v in (sys.argv[1:] or ["0"])]
    dev = torch.device("cuda")
    autotune.load_cache()
    m = create_model("resnet50", device=dev, compute_dtype="bf16" if str(dev).startswith("cuda") else None)
    m.ps.repack()
    probs = []
    seen = set()
    N = 64
    for l in m.all_layers():
        if not isinstance(l, ConvBN) or not hasattr(l, "pack") or l.name == "conv0":
            continue
        s = l.spec
        key = (l.in_shape, l.out_shape, s.kh, s.sh)
        if key in seen:
            continue
        seen.add(key)
        H, W, C = l.in_shape
        P, Q, K = l.out_shape
        x = torch.randn(N, H, W, C, device=dev).bfloat16()
        y = torch.empty(N, P, Q, K, device=dev, dtype=torch.bfloat16)
        acc = torch.zeros(16 * K, device=dev)
        probs.append((f"{l.name} fwd", lambda x=x, y=y, l=l, acc=acc: Fn.conv_forward(x, l.spec, l.pack.pack, None, y,
                                                                                    stats=acc, stats_R=8),
                      2.0 * N * P * Q * K * s.kh * s.kw * C))
        if l.need_dx:
            dz = torch.randn(N, P, Q, K, device=dev).bfloat16()
            dx = torch.zeros(N, H, W, C, device=dev, dtype=torch.bfloat16)
            probs.append((f"{l.name} dgrad", lambda dz=dz, dx=dx, l=l: Fn.conv_dgrad(dz, l.spec, l.pack.tr, None, dx,
                                                                                   False),
                          2.0 * N * P * Q * K * s.kh * s.kw * C))
            # the data-grad GEMM with the fused BN-backward epilogue (mode 1: ReLU mask from y,
            # beta-accumulate), as in the model
            z = torch.randn(N, H, W, C, device=dev).bfloat16()
            yv = torch.randn(N, H, W, C, device=dev).bfloat16()
            st = [torch.rand(C, device=dev) + 0.5 for _ in range(4)]
            bacc = torch.zeros(16 * C, device=dev)
            bnb = Fn.BNBwdFuse(z, yv, Fn.BNSaved(st[0], st[1]), st[2], st[3], 1, bacc, 8)
            probs.append((f"{l.name} dgrad+bnb", lambda dz=dz, dx=dx, l=l, bnb=bnb: Fn.conv_dgrad(
                dz, l.spec, l.pack.tr, None, dx, True, bnb=bnb), 2.0 * N * P * Q * K * s.kh * s.kw * C))
    # big GEMM probe, cfg 13 / 15
    Mb, Nb, Kb = 32768, 4096, 4096
    spec = Fn.ConvSpec(cin=Kb, cin_pad=Kb, cout=Nb, kh=1, kw=1)
    ps = ParamStore(seed=0)
    p = ps.add("w", (Nb, 1, 1, Kb), True, ps.variance_scaling(Kb))
    pk = ps.add_pack(p, Nb, 1, 1, Kb, spec.Kpad, spec.Kpad_t, want_tr=False)
    ps.finalize(dev)
    ps.repack()
    xb = torch.randn(Mb // 64, 8, 8, Kb, device=dev).bfloat16()
    yb = torch.empty(Mb // 64, 8, 8, Nb, device=dev, dtype=torch.bfloat16)
    for cfg in (13, 14, 15):
        probs.append((f"gemm32768x4096x4096 cfg{cfg}", lambda cfg=cfg: Fn.conv_forward(xb, spec, pk.pack, None, yb,
                                                                                     cfg=cfg), 2.0 * Mb * Nb * Kb))
    hcb = _ext.ops()

    def set_variant(v):  # the selector exists only in experiment builds
        try:
            hcb.set_igemm_variant(v)
        except (AttributeError, RuntimeError):
            if v != 0:
                raise SystemExit("this build has no hcb.set_igemm_variant; run with variant 0 only")

    res = {(n, v): [] for n, _, _ in probs for v in variants}
    for rnd in range(5):
        for v in variants:
            set_variant(v)
            for n, fn, fl in probs:
                res[(n, v)].append(t_us(fn))
    tot = {v: 0.0 for v in variants}
    print(f"{'problem':44s} " + " ".join(f"{'var' + str(v) + ' us':>10s}" for v in variants) + "   TF(best)")
    for n, _, fl in probs:
        meds = [statistics.median(res[(n, v)]) for v in variants]
        if not n.startswith("gemm"):
            for v, mv in zip(variants, meds):
                tot[v] += mv
        print(f"{n:44s} " + " ".join(f"{mv:10.1f}" for mv in meds) + f"   {fl / min(meds) / 1e6:6.0f}")
    print("sum over distinct ResNet-50 layers (us): " + "  ".join(f"var{v}={tot[v]:.1f}" for v in variants))


if __name__ == "__main__":
    main()
