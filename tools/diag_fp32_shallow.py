#!/usr/bin/env python3
"""fp32 shallow-net gradient check (tests/test_determinism_gpu.py's first half) with every
tensor printed, for the Trainer built with and without graphs, after optional pre-steps:
    python tools/diag_fp32_shallow.py [--bf16-first]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch

from azure_hc_intel_tf_amd.ops import functional as Fn
from azure_hc_intel_tf_amd.trainer import Trainer, constant_lr, synthetic_batch
from test_determinism_gpu import _grad_errors, _shallow


def main():
    kw = dict(image_size=32, image_channels=8, seed=5, num_classes=11)
    mc = _shallow("cpu", **kw)
    img_c, lab_c = synthetic_batch(mc, 32, seed=7)
    img_c = ((img_c - 127.0) / 60.0).to(torch.bfloat16).float()
    tc = Trainer(mc, 32, constant_lr(0.0), weight_decay=0.0)
    tc._forward_backward(img_c, lab_c)
    if "--bf16-first" in sys.argv:
        mg = _shallow("cuda", **kw)
        tg = Trainer(mg, 32, constant_lr(0.0), weight_decay=0.0, use_graph=False)
        tg._forward_backward(img_c.to("cuda", torch.bfloat16), lab_c.cuda())
    for graph in (False, True, False):
        mf = _shallow("cuda", compute_dtype="fp32", **kw)
        tf = Trainer(mf, 32, constant_lr(0.0), weight_decay=0.0, use_graph=graph)
        tf._forward_backward(img_c.cuda(), lab_c.cuda())
        torch.cuda.synchronize()
        print(f"== use_graph={graph} native={mf.native} f32_native={Fn._F32_NATIVE[0]} det={Fn.deterministic()}")
        for err, rel, cos, name in _grad_errors(mf, mc):
            print(f"   {name:40s} err {err:.2e} rel {rel:.2e} cos {cos}")


if __name__ == "__main__":
    main()
