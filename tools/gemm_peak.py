#!/usr/bin/env python3
"""Peak check of the implicit-GEMM conv kernels on a large plain GEMM (a 1x1 conv with
M = N*H*W rows): every tile config vs hipBLASLt (torch.matmul) on the same bf16 problem.
Separates kernel quality from the small-problem occupancy limits of the ResNet layers.

    python tools/gemm_peak.py [--M 32768 --N 4096 --K 4096]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from azure_hc_intel_tf_amd.nn.params import ParamStore
from azure_hc_intel_tf_amd.ops import functional as Fn
from azure_hc_intel_tf_amd.ops.autotune import _time


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=32768)
    ap.add_argument("--N", type=int, default=4096)
    ap.add_argument("--K", type=int, default=4096)
    a = ap.parse_args()
    dev = torch.device("cuda")
    spec = Fn.ConvSpec(cin=a.K, cin_pad=a.K, cout=a.N, kh=1, kw=1)
    ps = ParamStore(seed=0)
    p = ps.add("w", (a.N, 1, 1, a.K), True, ps.variance_scaling(a.K))
    pk = ps.add_pack(p, a.N, 1, 1, a.K, spec.Kpad, spec.Kpad_t, want_tr=False)
    ps.finalize(dev)
    ps.repack()
    x = torch.randn(a.M // 64, 8, 8, a.K, device=dev).bfloat16()
    y = torch.empty(a.M // 64, 8, 8, a.N, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * a.M * a.N * a.K
    xm, wm = x.view(a.M, a.K), pk.pack.view(a.N, -1)[:, :a.K]
    t = _time(lambda: xm @ wm.t(), reps=10) * 1000
    print(f"hipBLASLt (torch.matmul)  {t:8.1f} us {fl / t / 1e6:6.0f} TF", flush=True)
    for cfg in range(17):
        t = _time(lambda: Fn.conv_forward(x, spec, pk.pack, None, y, cfg=cfg), reps=10) * 1000
        print(f"conv cfg {cfg:2d} {str(Fn._CONV_TILES[cfg]):12s} {t:8.1f} us {fl / t / 1e6:6.0f} TF", flush=True)


if __name__ == "__main__":
    main()
