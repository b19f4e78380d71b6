#!/usr/bin/env python3
"""Where does the fused BN-backward data-grad epilogue lose time? For a few ResNet-50 bs64
data-grad problems: plain GEMM, + beta-accumulate, + BN-backward gating/sums (mode 2: mask
recomputed from z; mode 1: mask read from y), per tile config, against torch streaming
kernels moving the same bytes (achievable-bandwidth reference)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from azure_hc_intel_tf_amd.ops import autotune
from azure_hc_intel_tf_amd.ops import functional as Fn
from azure_hc_intel_tf_amd.ops.functional import ConvSpec
from azure_hc_intel_tf_amd.nn.params import ParamStore


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
    dev = "cuda"
    autotune.load_cache()
    # name, cin (dgrad N), cout (dgrad K), H, N
    probs = [("s1b2c1 256<-64", 256, 64, 56), ("s1c3 64<-256", 64, 256, 56), ("s2b2c1 512<-128", 512, 128, 28),
             ("s3b2c1 1024<-256", 1024, 256, 14), ("s3c3 256<-1024", 256, 1024, 14)]
    N = 64
    for name, cin, cout, H in probs:
        spec = ConvSpec(cin=cin, cin_pad=cin, cout=cout, kh=1, kw=1, sh=1, sw=1, pt=0, pl=0, pb=0, pr=0)
        ps = ParamStore(seed=0)
        p = ps.add("w", (cout, 1, 1, cin), True, ps.variance_scaling(cin, -1))
        pk = ps.add_pack(p, cout, 1, 1, cin, spec.Kpad, spec.Kpad_t, want_tr=True)
        ps.finalize(dev)
        ps.repack()
        dz = torch.randn(N, H, H, cout, device=dev).bfloat16()
        dx = torch.randn(N, H, H, cin, device=dev).bfloat16()
        z = torch.randn(N, H, H, cin, device=dev).bfloat16()
        y = torch.relu(torch.randn(N, H, H, cin, device=dev)).bfloat16()
        st = [torch.rand(cin, device=dev) + 0.5 for _ in range(4)]
        acc = torch.zeros(8 * 2 * cin, device=dev)
        M = N * H * H
        tuned = Fn._tuned.get(Fn.dgb_key(M, cin, cout, 1))
        mb = M * cin * 2 / 1e6
        print(f"== {name}: M={M} N={cin} K={cout}; dX tensor {mb:.1f} MB, dY {M * cout * 2 / 1e6:.1f} MB; tuned dgb cfg {tuned}")
        for cfg in sorted({tuned if isinstance(tuned, int) else 0, 0, 1, 2, 3, 5, 13}):
            r = {}
            r["plain"] = tm(lambda: Fn.conv_dgrad(dz, spec, pk.tr, p.data, dx, False, cfg=cfg))
            r["beta"] = tm(lambda: Fn.conv_dgrad(dz, spec, pk.tr, p.data, dx, True, cfg=cfg))
            for mode, acc_ in ((2, False), (1, False), (1, True)):
                bnb = Fn.BNBwdFuse(z, y, Fn.BNSaved(st[0], st[1]), st[2], st[3], mode, acc, 8)
                r[f"m{mode}{'+b' if acc_ else ''}"] = tm(
                    lambda: Fn.conv_dgrad(dz, spec, pk.tr, p.data, dx, acc_, cfg=cfg, bnb=bnb))
            print(f"  cfg {cfg:2d}: " + "  ".join(f"{k} {v:6.1f}" for k, v in r.items()), flush=True)
        a, b, c = dx, z, y
        o = torch.empty_like(a)
        t_copy = tm(lambda: o.copy_(a))
        t_add = tm(lambda: torch.add(a, b, out=o))
        t_3 = tm(lambda: torch.addcmul(a, b, c, out=o))
        # mb is MB and the times are us: MB / us = TB/s
        print(f"  torch stream: copy(1R1W) {t_copy:.1f} us = {2 * mb / t_copy:.2f} TB/s; add(2R1W) {t_add:.1f} "
              f"= {3 * mb / t_add:.2f} TB/s; addcmul(3R1W) {t_3:.1f} = {4 * mb / t_3:.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
