#!/usr/bin/env python3
"""Library reference point for the 1x1-conv GEMMs of ResNet-50 (bs=64): hipBLASLt via
torch.matmul on the same [M,K]x[K,N] bf16 problems as our implicit-GEMM kernels
(fwd: y[M,Cout] = x[M,Cin] W^T, dgrad: dx[M,Cin] = dy[M,Cout] W, wgrad: dW[Cout,Cin] = dy^T x).

    python tools/gemm_ref.py [--batch 64]
"""
import argparse
import json

import torch

SHAPES = [  # (H*W of the output, Cin, Cout) of every distinct 1x1 conv in ResNet-50 (stride folded into M)
    (3136, 64, 256), (3136, 64, 64), (3136, 256, 64), (784, 256, 512), (784, 256, 128), (784, 128, 512),
    (784, 512, 128), (196, 512, 1024), (196, 512, 256), (196, 256, 1024), (196, 1024, 256), (49, 1024, 2048),
    (49, 1024, 512), (49, 512, 2048), (49, 2048, 512),
]


def tm(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    rows = []
    for hw, cin, cout in SHAPES:
        M = a.batch * hw
        x = torch.randn(M, cin, device="cuda").bfloat16()
        w = torch.randn(cout, cin, device="cuda").bfloat16()
        dy = torch.randn(M, cout, device="cuda").bfloat16()
        fl = 2.0 * M * cin * cout
        t_f = tm(lambda: x @ w.t())
        t_d = tm(lambda: dy @ w)
        t_w = tm(lambda: dy.t() @ x)
        r = {"M": M, "cin": cin, "cout": cout, "fwd_us": t_f, "dgrad_us": t_d, "wgrad_us": t_w,
             "fwd_tf": fl / t_f / 1e6, "dgrad_tf": fl / t_d / 1e6, "wgrad_tf": fl / t_w / 1e6}
        rows.append(r)
        print(f"M={M:7d} {cin:5d}->{cout:5d}  fwd {t_f:6.1f}us ({r['fwd_tf']:4.0f}TF)  dgrad {t_d:6.1f}us "
              f"({r['dgrad_tf']:4.0f}TF)  wgrad {t_w:6.1f}us ({r['wgrad_tf']:4.0f}TF)", flush=True)
    print(json.dumps({"rows": rows}))


if __name__ == "__main__":
    main()
