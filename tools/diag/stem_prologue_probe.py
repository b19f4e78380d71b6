#!/usr/bin/env python3
"""Bitwise probe of the ResNet stem's BN + ReLU + max-pool kernel (bn.hip bn_relu_maxpool_acc_kernel)
across two builds of the kernel library (the LDS-coefficient prologue of commit
d89ce99 made tests/test_determinism_gpu.py's trajectory check fail; is that a bug or rounding?).

    HCB_KERNELS_SO=<lib A> python tools/diag/stem_prologue_probe.py run gpurun_out/stemA.pt
    HCB_KERNELS_SO=<lib B> python tools/diag/stem_prologue_probe.py run gpurun_out/stemB.pt
    python tools/diag/stem_prologue_probe.py compare gpurun_out/stemA.pt gpurun_out/stemB.pt

``run`` feeds the kernel the determinism test's stem shape (bs 16, 96 px -> z [16, 48, 48, 64],
3x3/2 pool) from a fixed seed, once with the training replica count (R = 8: the kernel's
straight-line replica loads) and once with the deterministic mode's one-replica-per-64-rows
(R = 576: the generic replica loop), for the bf16 build (bf16 y) and the fp32 path (planes y), and
saves y, the argmax, the saved mean / invstd and the running statistics. ``compare`` reports, per
output, how many elements differ and the largest difference in units in the last place."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch


def run(out_path):
    from azure_hc_intel_tf_amd.nn.layers import set_gpu_compute_dtype
    from azure_hc_intel_tf_amd.ops import functional as Fn

    dev = "cuda"
    N, H, C, P = 16, 48, 64, 24
    res = {}
    for path in ("bf16", "fp32"):
        if path == "fp32":
            set_gpu_compute_dtype(torch.float32)
            Fn.set_f32_native(True)
        g = torch.Generator().manual_seed(21)
        zf = (torch.randn(N, H, H, C, generator=g) * 2.0 + 0.3)
        z = zf.to(dev, torch.float32 if path == "fp32" else torch.bfloat16)
        gamma = (torch.rand(C, generator=g) + 0.5).to(dev)
        beta = (torch.randn(C, generator=g) * 0.1).to(dev)
        shift = (torch.randn(C, generator=g) * 0.1).to(dev)
        M = N * H * H
        v = (z.float() - shift).view(M, C)
        for R in (8, (M + 63) // 64):
            # replica r holds the sums of rows r, r + R, ... (fixed, exact-order CPU sums in fp64 -> fp32)
            acc = torch.zeros(R, 2, C, dtype=torch.float64)
            vc = v.double().cpu()
            for r in range(R):
                acc[r, 0] = vc[r::R].sum(0)
                acc[r, 1] = (vc[r::R] ** 2).sum(0)
            acc = acc.float().to(dev)
            out = Fn.Planes.empty((N, P, P, C), dev) if path == "fp32" else torch.empty(N, P, P, C, dtype=z.dtype,
                                                                                        device=dev)
            amax = torch.empty(N, P, P, C, dtype=torch.uint8, device=dev)
            sm, si = torch.empty(C, device=dev), torch.empty(C, device=dev)
            rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
            Fn.bn_relu_maxpool_acc(z, gamma, beta, rm, rv, 0.9, 1e-5, acc, R, sm, si, out, amax, 3, 3, 2, 2,
                                   (0, 1, 0, 1), shift=shift)
            torch.cuda.synchronize()
            key = f"{path}_R{R}"
            res[key + "_y"] = (out.float() if path == "fp32" else out.float()).cpu()
            res[key + "_amax"] = amax.cpu()
            res[key + "_mean"] = sm.cpu()
            res[key + "_invstd"] = si.cpu()
            res[key + "_rmean"] = rm.cpu()
            res[key + "_rvar"] = rv.cpu()
        if path == "fp32":
            Fn.set_f32_native(False)
            set_gpu_compute_dtype(torch.bfloat16)
    torch.save(res, out_path)
    print(f"saved {len(res)} tensors to {out_path} (library {os.environ.get('HCB_KERNELS_SO', 'in-tree')})")


def ulps(a, b):
    if a.dtype == torch.uint8:
        return int((a != b).sum()), 0
    ai = a.float().contiguous().view(torch.int32).long()
    bi = b.float().contiguous().view(torch.int32).long()
    # map the sign-magnitude float order onto integers
    ai = torch.where(ai < 0, -(ai & 0x7FFFFFFF), ai)
    bi = torch.where(bi < 0, -(bi & 0x7FFFFFFF), bi)
    d = (ai - bi).abs()
    return int((d > 0).sum()), int(d.max())


def compare(pa, pb):
    a, b = torch.load(pa, weights_only=True), torch.load(pb, weights_only=True)
    worst = 0
    for k in sorted(a):
        n, u = ulps(a[k], b[k])
        if k.startswith("bf16_") and k.endswith("_y"):
            u //= 65536  # bf16 values: ulps of bf16
        worst = max(worst, u)
        print(f"{k:24s} {tuple(a[k].shape)!s:22s} differing {n:8d} / {a[k].numel():8d}   max ulp {u}")
    print(f"largest difference: {worst} ulp")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        compare(sys.argv[2], sys.argv[3])
