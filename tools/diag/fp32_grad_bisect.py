"""Diagnostic: per-parameter gradient error of one fp32 GPU step (plane GEMMs) vs the fp32 CPU step,
with fusion switches toggled (bisects a backward discrepancy to a layer / feature)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.nn import layers as L
from azure_hc_intel_tf_amd.ops import functional as Fn
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch


def run(label, **switches):
    for k, v in switches.items():
        setattr(L if hasattr(L, k) else Fn, k, v)
    kw = dict(image_size=64, seed=7, image_channels=8)
    mg = create_model("resnet50", device="cuda", compute_dtype="fp32", **kw)
    mc = create_model("resnet50", device="cpu", **kw)
    img_c, lab_c = synthetic_batch(mc, 4, seed=3)
    img_c = (img_c - 127.0) / 60.0
    tg = Trainer(mg, 4, constant_lr(0.05), use_graph=False)
    tc = Trainer(mc, 4, constant_lr(0.05))
    lg = float(tg.step(img_c.cuda(), lab_c.cuda()))
    lc = float(tc.step(img_c, lab_c))
    gg, gc = mg.ps.grad.cpu(), mc.ps.grad
    print(f"== {label}: loss {lg:.7f} vs {lc:.7f}; grad rel {float((gg - gc).norm() / gc.norm()):.3e}")
    worst = []
    for p in mc.ps.params:
        a = gg[p.offset:p.offset + p.numel]
        b = gc[p.offset:p.offset + p.numel]
        worst.append((float((a - b).norm() / (b.norm() + 1e-30)), p.name))
    for e, n in worst[:12] + sorted(worst, reverse=True)[:8]:
        print(f"   {n:45s} {e:.3e}")
    Fn.set_f32_native(False)
    from azure_hc_intel_tf_amd.nn.layers import set_gpu_compute_dtype
    set_gpu_compute_dtype(torch.bfloat16)
    for k in switches:
        setattr(L if hasattr(L, k) else Fn, k, DEFAULTS[k])


DEFAULTS = {"FUSE_BN_BWD": True, "STEM_S2D": True}
run("default")
run("no fused BN backward", FUSE_BN_BWD=False)
run("direct stem", STEM_S2D=False)
