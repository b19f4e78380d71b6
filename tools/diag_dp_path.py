#!/usr/bin/env python3
"""Loss trace of the multi-GPU step path forced onto one GPU (segmented graphs + async RCCL
engine on a 1-rank communicator) vs the single-graph step, ResNet-50 bs=64 224px.

    python tools/diag_dp_path.py [--compression bf16] [--steps 12]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.ops import autotune
from azure_hc_intel_tf_amd.parallel.native import NativeReducer
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, resnet_lr_schedule, synthetic_batch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--compression", default=None)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--graph", type=int, default=1)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--schedule", action="store_true", help="bench.py's ResNet lr schedule instead of --lr")
    ap.add_argument("--modes", default="single,dp")
    ap.add_argument("--nosync", action="store_true", help="device-side loss trace, no host sync between steps")
    ap.add_argument("--reducer_first", action="store_true", help="create the communicator before the model")
    a = ap.parse_args()
    autotune.load_cache()
    for mode in a.modes.split(","):
        torch.manual_seed(0)
        red = NativeReducer(compression=a.compression, force=True) if (mode == "dp" and a.reducer_first) else None
        m = create_model("resnet50", device="cuda", compute_dtype="bf16")
        img, lab = synthetic_batch(m, 64)
        if mode == "dp" and red is None:
            red = NativeReducer(compression=a.compression, force=True)
        t = Trainer(m, 64, resnet_lr_schedule(64) if a.schedule else constant_lr(a.lr), reducer=red, world_size=1, use_graph=bool(a.graph),
                    force_overlap=mode == "dp")
        out = []
        if a.nosync:
            tr = torch.zeros(a.steps, device="cuda")
            for i in range(a.steps):
                tr[i:i + 1].copy_(t.step(img, lab))
            out = [round(v, 4) for v in tr.tolist()]
        else:
            for _ in range(a.steps):
                out.append(float(t.step(img, lab)))
                g = m.ps.grad
                out[-1] = (round(out[-1], 4), round(float(g.abs().max()), 4), bool(torch.isfinite(g).all()))
        print(mode, "nosync" if a.nosync else "sync", "reducer_first" if a.reducer_first else "", out, flush=True)
        if red is not None:
            red.close()


if __name__ == "__main__":
    main()
