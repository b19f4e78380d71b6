#!/usr/bin/env python3
"""Autotune every conv GEMM problem of the BASELINE model configs on this GPU and write the
in-tree cache (azure_hc_intel_tf_amd/tuned/mi355x.json): resnet50 bs64 / bs256, resnet152
bs128, inception3 bs64, resnet101 bs64, resnet50_v1.5 bs64. A copy goes to gpurun_out/.

    python tools/tune_all.py [--dtype bf16|fp32|both] [model ...]

(fp32: the bf16-plane GEMM problems of the models' fp32 path, keys fwd3 / wgrad3.)"""
import os
import shutil
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.ops import autotune

CONFIGS = [("resnet50", 64), ("resnet50", 256), ("resnet152", 128), ("inception3", 64), ("resnet101", 64),
           ("resnet50_v1.5", 64)]


def main():
    args = sys.argv[1:]
    dtypes = ["bf16"]
    if "--dtype" in args:
        i = args.index("--dtype")
        dtypes = ["bf16", "fp32"] if args[i + 1] == "both" else [args[i + 1]]
        del args[i:i + 2]
    only = args
    autotune.load_cache()
    for dt in dtypes:
        for name, b in CONFIGS:
            if only and name not in only:
                continue
            t0 = time.time()
            m = create_model(name, device="cuda", compute_dtype=None if dt == "bf16" else dt)
            n = autotune.tune_model(m, b, verbose=True, save=True)  # per-layer lines: progress for gpurun
            del m
            torch.cuda.empty_cache()
            print(f"{name} {dt} bs{b}: tuned {n} problems in {time.time() - t0:.0f} s", flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    shutil.copy(autotune.DEFAULT_CACHE, "gpurun_out/mi355x.json")


if __name__ == "__main__":
    main()
