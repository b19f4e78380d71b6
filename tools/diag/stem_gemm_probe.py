#!/usr/bin/env python3
"""The fp32 S2D stem GEMM (M = N x 112 x 112, N = 64, K = 256 row windows) in isolation, per cfg:
time (HIP events) -- a target for rocprofv3 --pmc passes too.

    python tools/diag/stem_gemm_probe.py [--cfgs 19,33,34,35] [--reps 30]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from azure_hc_intel_tf_amd.models import create_model  # noqa: E402
from azure_hc_intel_tf_amd.nn.layers import StemS2D  # noqa: E402
from azure_hc_intel_tf_amd.ops import autotune  # noqa: E402
from azure_hc_intel_tf_amd.ops import functional as Fn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="19,33,34,35,20,18")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    dev = torch.device("cuda")
    m = create_model("resnet50", device=dev, compute_dtype="fp32")
    m.ps.repack()
    autotune.load_cache()
    st = [l for l in m.all_layers() if isinstance(l, StemS2D)][0]
    N = a.batch
    x = torch.randn(N, 224, 224, st.in_shape[2], device=dev)
    xf = st.fold_input(x)
    P, Q, C = st.out_shape
    z = torch.empty(N, P, Q, C, device=dev)
    R = 8
    acc = torch.zeros(R * 2 * C, device=dev)
    w = st._folded_weight(dev)
    for c in [int(v) for v in a.cfgs.split(",")]:
        fn = lambda: Fn.conv_forward(xf, st.fold_spec, w, st.w.data, z, stats=acc, stats_R=R, cfg=(c, 1))
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) / a.reps * 1000
        fl = 2.0 * N * P * Q * C * 256
        print(f"stem fwd cfg={c} {us:.1f} us  {fl / us / 1e6:.0f} TF (x6 MFMA: {6 * fl / us / 1e6 / 25:.0f}% of 2.5 PF)",
              flush=True)


if __name__ == "__main__":
    main()
