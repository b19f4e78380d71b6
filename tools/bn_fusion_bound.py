#!/usr/bin/env python3
"""Upper bound of fusing the bottleneck conv1 / conv2 BatchNorm apply into the consuming convs
(VERDICT round 2, next step 1): the ResNet-50 bs=64 training step timed with those 32 apply
passes simply SKIPPED (the conv output is handed on as the activation -- numerically wrong, a
timing bound only) against the real step, in alternating runs. Whatever a fused consumer costs
(BN parameters staged per block, a transform of every loaded A / X vector, halo masking) has to
come out of this difference.

    python tools/bn_fusion_bound.py --skip 0|1 --steps 40 --warmup 10
prints one JSON line {"skip": ..., "ms_per_step": ...}"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import azure_hc_intel_tf_amd  # noqa: E402,F401


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=10)
    a = ap.parse_args()
    import torch

    from azure_hc_intel_tf_amd.models import create_model
    from azure_hc_intel_tf_amd.nn import layers as L
    from azure_hc_intel_tf_amd.ops import _ext, autotune
    from azure_hc_intel_tf_amd.ops import functional as Fn
    from azure_hc_intel_tf_amd.trainer import Trainer, resnet_lr_schedule, synthetic_batch

    if a.skip:
        orig = L.ConvBN.forward

        def forward(self, x, out=None, residual=None, residual_bn=None):
            if (self.bn and self.relu and residual is None and self.training and Fn.native(x)
                    and self.name.rsplit("/", 1)[-1] in ("conv1", "conv2")):
                N = x.shape[0]
                P, Q, C = self.out_shape
                z = L.empty_act((N, P, Q, C), x.device)
                x = self._conv_fwd_stats(x, z)
                self._saved = (x, z, z, Fn.BNSaved(self.sv_mean.data, self.sv_invstd.data), False)
                return z
            return orig(self, x, out, residual, residual_bn)

        L.ConvBN.forward = forward
    _ext.load()
    dev = torch.device("cuda", 0)
    m = create_model("resnet50", device=dev, compute_dtype="bf16")
    autotune.load_cache()
    autotune.tune_model(m, 64, save=False)
    img, lab = synthetic_batch(m, 64)
    t = Trainer(m, 64, resnet_lr_schedule(64))
    for _ in range(a.warmup):
        t.step(img, lab)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        t.step(img, lab)
    torch.cuda.synchronize()
    ms = 1000.0 * (time.perf_counter() - t0) / a.steps
    print(json.dumps({"skip": a.skip, "ms_per_step": round(ms, 4), "img_per_s": round(64000.0 / ms, 1)}), flush=True)


if __name__ == "__main__":
    main()
