#!/usr/bin/env python3
"""Per-layer timing of the hand-written conv kernels (fwd / dgrad / wgrad) of a model, with
MIOpen (torch conv, channels_last bf16) timed on the same shapes as a comparison point.

    python tools/conv_bench.py --model resnet50 --batch 64 [--no_miopen] [--tune] [--fp32]

--fp32: the reference-precision kernels (bf16-plane operands, bf16x6 GEMMs, conv_p3.hip) at their
tuned configs; TF columns are fp32 FLOP/s and "mfma%" the share of the 2.5 PF bf16 dense peak the
six MFMA products run at.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.nn.layers import ConvBN
from azure_hc_intel_tf_amd.ops import autotune
from azure_hc_intel_tf_amd.ops import functional as Fn


def tm(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1000.0  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--no_miopen", action="store_true")
    ap.add_argument("--tune", action="store_true")
    ap.add_argument("--json", default=None)
    ap.add_argument("--fp32", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda")
    m = create_model(a.model, device=dev, compute_dtype="fp32" if a.fp32 else None)
    if a.fp32:
        a.no_miopen = True
    m.ps.repack()
    autotune.load_cache()
    if a.tune:
        autotune.tune_model(m, a.batch, save=False)
    seen = {}
    rows = []
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0, "mi_fwd": 0.0, "mi_dgrad": 0.0, "mi_wgrad": 0.0}
    for l in m.all_layers():
        if not isinstance(l, ConvBN):
            continue
        s = l.spec
        key = (l.in_shape, l.out_shape, s.kh, s.kw, s.sh, s.pt, l.need_dx)
        if key in seen:
            seen[key]["count"] += 1
            r = seen[key]
            for k in ("fwd", "dgrad", "wgrad"):
                tot[k] += r[k]
                if r.get("mi_" + k) is not None:
                    tot["mi_" + k] += r["mi_" + k]
            continue
        N = a.batch
        H, W, C = l.in_shape
        P, Q, K = l.out_shape
        if a.fp32:
            m.activate()
            x = Fn.to_planes(torch.randn(N, H, W, C, device=dev))
            dz = Fn.to_planes(torch.randn(N, P, Q, K, device=dev))
            y = torch.empty(N, P, Q, K, device=dev)
        else:
            x = torch.randn(N, H, W, C, device=dev).bfloat16()
            dz = torch.randn(N, P, Q, K, device=dev).bfloat16()
            y = torch.empty(N, P, Q, K, device=dev, dtype=torch.bfloat16)
        slab, T, cfg = Fn.conv_stats_slab(x.shape, s, dev)
        r = {"layer": l.name, "in": list(l.in_shape), "out": list(l.out_shape), "k": [s.kh, s.kw], "stride": s.sh,
             "count": 1}
        acc = torch.zeros(8 * 2 * K, device=dev)
        r["fwd"] = tm(lambda: Fn.conv_forward(x, s, l.pack.pack, None, y, stats=acc, stats_R=8))
        dw = torch.zeros(K, s.K, device=dev)
        r["wgrad"] = tm(lambda: Fn.conv_wgrad(dz, x, s, dw))
        if l.need_dx:
            dx = torch.zeros(N, H, W, C, device=dev, dtype=torch.float32 if a.fp32 else torch.bfloat16)
            r["dgrad"] = tm(lambda: Fn.conv_dgrad(dz, s, l.pack.tr, None, dx, False))
        else:
            r["dgrad"] = 0.0
        flops = 2.0 * N * P * Q * K * s.kh * s.kw * s.cin
        r["gflop"] = flops / 1e9
        r["tf_fwd"] = flops / r["fwd"] / 1e6
        r["tf_wgrad"] = flops / r["wgrad"] / 1e6
        r["tf_dgrad"] = flops / r["dgrad"] / 1e6 if r["dgrad"] else None
        if not a.no_miopen and s.cin % 8 == 0 and s.cin == s.cin_pad:
            xt = x.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last).requires_grad_(True)
            wt = torch.randn(K, C, s.kh, s.kw, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
            wt.requires_grad_(True)
            pad = (s.pt, s.pl) if (s.pt == s.pb and s.pl == s.pr) else None
            if pad is not None:
                fw = lambda: F.conv2d(xt, wt, stride=s.sh, padding=pad)
                r["mi_fwd"] = tm(fw)
                out = fw()
                go = torch.randn_like(out)
                r["mi_dgrad"] = tm(lambda: torch.ops.aten.convolution_backward(
                    go, xt, wt, None, (s.sh, s.sw), pad, (1, 1), False, (0, 0), 1, (True, False, False)))
                r["mi_wgrad"] = tm(lambda: torch.ops.aten.convolution_backward(
                    go, xt, wt, None, (s.sh, s.sw), pad, (1, 1), False, (0, 0), 1, (False, True, False)))
                for k in ("fwd", "dgrad", "wgrad"):
                    tot["mi_" + k] += r["mi_" + k]
        for k in ("fwd", "dgrad", "wgrad"):
            tot[k] += r[k]
        seen[key] = r
        rows.append(r)
        if a.fp32:
            M = N * P * Q
            r["cfg"] = [Fn.p3_plan(M, K, s.K, s.kh * s.kw), Fn.wgrad_p3_plan(K, s.K, M, s.kh * s.kw)]
            pk = lambda t: f"{6 * flops / t / 1e6 / 2500 * 100:4.0f}%" if t else "   -"
            print(f"{l.name:28s} {str(l.in_shape):16s}->{str(l.out_shape):16s} k{s.kh}x{s.kw}/{s.sh} "
                  f"fwd {r['fwd']:7.1f}us ({r['tf_fwd']:4.0f}TF {pk(r['fwd'])}) | dgrad {r['dgrad']:7.1f}us "
                  f"({pk(r['dgrad'])}) | wgrad {r['wgrad']:7.1f}us ({r['tf_wgrad']:4.0f}TF {pk(r['wgrad'])}) "
                  f"cfg {r['cfg']}", flush=True)
        else:
            mi = lambda k: f"{r.get('mi_' + k, 0) or 0:7.1f}"
            print(f"{l.name:28s} {str(l.in_shape):16s}->{str(l.out_shape):16s} k{s.kh}x{s.kw}/{s.sh} "
                  f"fwd {r['fwd']:7.1f}us ({r['tf_fwd']:5.0f}TF) mi {mi('fwd')} | "
                  f"dgrad {r['dgrad']:7.1f} mi {mi('dgrad')} | wgrad {r['wgrad']:7.1f}us ({r['tf_wgrad']:5.0f}TF) "
                  f"mi {mi('wgrad')}", flush=True)
    print("TOTAL per step (us): " + json.dumps({k: round(v, 1) for k, v in tot.items()}))
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"rows": rows, "total_us": tot}, f, indent=1)


if __name__ == "__main__":
    main()
