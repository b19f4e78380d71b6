#!/usr/bin/env python3
"""Shortcut-BN reduction fused into the dgrad epilogue (FUSE_RES_BN_BWD) against the unfused pass:
per-parameter gradient norms / relative differences of the shortcut BNs and the whole gradient,
bf16 and fp32, default and deterministic mode."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.nn import layers as L
from azure_hc_intel_tf_amd.nn.layers import set_gpu_compute_dtype
from azure_hc_intel_tf_amd.ops import functional as Fn
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch


def run(dtype, fuse, det):
    L.FUSE_RES_BN_BWD = fuse
    Fn.set_deterministic(det)
    m = create_model("resnet50", image_size=64, device="cuda", seed=11, compute_dtype=None if dtype == "bf16" else "fp32")
    img, lab = synthetic_batch(m, 8, seed=2)
    if dtype == "fp32":
        img[..., :3] = (img[..., :3] - 127.0) / 60.0
    t = Trainer(m, 8, constant_lr(0.0), weight_decay=0.0, use_graph=False)
    t._forward_backward(img, lab)
    torch.cuda.synchronize()
    g = {p.name: p.grad.float().cpu().clone() for p in m.ps.params}
    Fn.set_f32_native(False)
    set_gpu_compute_dtype(torch.bfloat16)
    Fn.set_deterministic(False)
    return g


for dtype in ("bf16", "fp32"):
    for det in (False, True):
        a, b, c = run(dtype, False, det), run(dtype, True, det), run(dtype, False, det)
        print(f"== {dtype} det={det}")
        for name in a:
            if "shortcut/batchnorm" in name or name.startswith("stage1/block1/conv3/batchnorm"):
                r = ((b[name] - a[name]).norm() / a[name].norm()).item()
                r0 = ((c[name] - a[name]).norm() / a[name].norm()).item()
                print(f"  {name:45s} |g| {a[name].norm().item():.4e} fused-vs-unfused {r:.3e}  unfused-rerun {r0:.3e}"
                      f"  first {a[name][:3].tolist()} / {b[name][:3].tolist()}")
