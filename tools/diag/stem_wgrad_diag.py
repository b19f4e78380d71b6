"""Diagnostic: the fp32 S2D stem's folded weight gradient inside a model step vs fp64."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import torch.nn.functional as F

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.nn.layers import StemS2D
from azure_hc_intel_tf_amd.ops import functional as Fn
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch

cap = {}
orig = StemS2D._wgrad


def spy(self, dz, x):
    cap["dz"] = dz.float().clone() if Fn.is_planes(dz) else dz.float().clone()
    cap["x"] = x.float().clone() if Fn.is_planes(x) else x.float().clone()
    dwf = torch.zeros((self.spec.cout, 256), dtype=torch.float32, device=dz.device)
    Fn.conv_wgrad(dz, x, self.fold_spec, dwf)
    cap["dwf"] = dwf.clone()
    cap["plan"] = Fn.wgrad_p3_plan(self.spec.cout, 256, dz.shape[0] * dz.shape[1] * dz.shape[2], 16)
    return orig(self, dz, x)


StemS2D._wgrad = spy
for bs, size in ((4, 64), (2, 64), (8, 64)):
    m = create_model("resnet50", device="cuda", compute_dtype="fp32", image_size=size, seed=7)
    img, lab = synthetic_batch(m, bs, seed=3)
    img = (img - 127.0) / 60.0
    t = Trainer(m, bs, constant_lr(0.05), use_graph=False)
    t.step(img, lab)
    torch.cuda.synchronize()
    dz, xf = cap["dz"].double(), cap["x"].double()  # [N,P,Q,64], [N,P+3,Q+3,16]
    ref = torch.nn.grad.conv2d_weight(xf.permute(0, 3, 1, 2), (64, 16, 4, 4), dz.permute(0, 3, 1, 2))
    ref = ref.permute(0, 2, 3, 1).reshape(64, 256)
    got = cap["dwf"].double()
    print(f"bs {bs} {size}px plan {cap['plan']} dz {tuple(dz.shape)} xf {tuple(xf.shape)}: "
          f"rel {float((got - ref).norm() / ref.norm()):.3e}")
    # which columns are wrong
    colerr = ((got - ref).norm(dim=0) / (ref.norm(dim=0) + 1e-30))
    print("  worst cols", [(int(i), round(float(colerr[i]), 4)) for i in colerr.argsort(descending=True)[:8]])
    Fn.set_f32_native(False)
