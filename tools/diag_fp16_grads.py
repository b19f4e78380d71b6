#!/usr/bin/env python3
"""Per-parameter gradient agreement of one training step: bf16 kernel build vs IEEE-fp16 build
(same weights, same batch, static loss scale)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch


def main():
    model = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    out = {}
    for dt in ("bf16", "fp16"):
        m = create_model(model, image_size=64, device="cuda", compute_dtype=dt, seed=11)
        img, lab = synthetic_batch(m, 8, seed=4)
        t = Trainer(m, 8, constant_lr(0.0), loss_scale=1024.0, use_graph=False)
        loss = float(t.step(img, lab))
        torch.cuda.synchronize()
        out[dt] = (loss, {p.name: p.grad.detach().double().cpu().clone() for p in m.ps.params})
    print("loss", out["bf16"][0], out["fp16"][0])
    rows = []
    for name, gb in out["bf16"][1].items():
        gh = out["fp16"][1][name]
        cos = float((gb.flatten() @ gh.flatten()) / (gb.norm() * gh.norm() + 1e-30))
        rows.append((cos, name, gb.norm().item(), gh.norm().item()))
    rows.sort()
    for r in rows[:25]:
        print(f"cos {r[0]:+.4f}  |g| bf16 {r[2]:.3e} fp16 {r[3]:.3e}  {r[1]}")
    print("...")
    for r in rows[-5:]:
        print(f"cos {r[0]:+.4f}  |g| bf16 {r[2]:.3e} fp16 {r[3]:.3e}  {r[1]}")


if __name__ == "__main__":
    main()
