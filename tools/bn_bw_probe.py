"""HBM throughput of the BN streaming passes against a plain copy, per ResNet-50 bs=64 BN shape.

  python tools/bn_bw_probe.py [--dtype bf16|fp32] [--graph]    (HCB_BN_BLOCKS=<n> sets the grid target)

Prints, per [M, C]: torch copy (1 read + 1 write), bn_apply_acc (read z, write y), bn_bwd_apply_acc
(read g + z, write dz), each as us and TB/s of the bytes it must move."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from azure_hc_intel_tf_amd.ops import _ext  # noqa: E402

SHAPES = [(200704, 64), (200704, 256), (50176, 128), (50176, 512), (12544, 256), (12544, 1024),
          (3136, 512), (3136, 2048), (802816, 64)]


GRAPH = False


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    if GRAPH:  # per-launch time inside a replayed graph (no host launch gaps)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
        g.replay()
        inner = g.replay
    else:
        inner = None
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    if inner is not None:
        inner()
    else:
        for _ in range(reps):
            fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--graph", action="store_true")
    a = ap.parse_args()
    global GRAPH
    GRAPH = a.graph
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    es = 2 if dt == torch.bfloat16 else 4
    hcb = _ext.ops()
    dev = "cuda"
    R = 8
    print(f"HCB_BN_BLOCKS={os.environ.get('HCB_BN_BLOCKS', 'default')} dtype={a.dtype} graph={a.graph}")
    print(f"{'M':>7} {'C':>5} {'MB':>6} | {'copy us':>8} {'TB/s':>5} | {'apply us':>8} {'TB/s':>5} | {'bwd us':>8} {'TB/s':>5}")
    for M, C in SHAPES:
        z = torch.randn(M, C, device=dev).to(dt)
        y = torch.empty_like(z)
        g = torch.randn_like(z)
        acc = torch.zeros(R, 2, C, device=dev)
        acc[:, 1] = float(M) / R
        gamma = torch.ones(C, device=dev)
        beta = torch.zeros(C, device=dev)
        sm, si = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        dgm, dbt = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        nb = M * C * es
        t_copy = timeit(lambda: y.copy_(z))
        t_ap = timeit(lambda: hcb.bn_apply_acc(z, C, y, C, None, 0, M, C, acc, R, 1e-5, 0.9, gamma, beta, 1, sm, si,
                                               None, None))
        t_bw = timeit(lambda: hcb.bn_bwd_apply_acc(g, C, None, 0, z, C, y, C, M, C, sm, si, gamma, beta, acc, R, dgm,
                                                   dbt, 0))
        print(f"{M:7d} {C:5d} {nb / 1e6:6.1f} | {t_copy:8.1f} {2 * nb / t_copy / 1e6:5.2f} | {t_ap:8.1f} "
              f"{2 * nb / t_ap / 1e6:5.2f} | {t_bw:8.1f} {3 * nb / t_bw / 1e6:5.2f}", flush=True)


if __name__ == "__main__":
    main()
