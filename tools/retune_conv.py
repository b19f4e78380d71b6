#!/usr/bin/env python3
"""Drop the forward / data-grad (plain and fused BN-backward) entries of the in-tree autotune
cache for the given model configs' problems and re-tune them (after a change to the conv
kernels' launch resources); weight-grad entries are kept. Default: resnet50 bs64 only.
--taps T: drop only the entries of T-tap filters (e.g. 9 after a change to the 3x3 kernels)."""
import os
import shutil
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from azure_hc_intel_tf_amd.models import create_model
from azure_hc_intel_tf_amd.ops import autotune
from azure_hc_intel_tf_amd.ops import functional as Fn
from tune_all import CONFIGS


def main():
    args = sys.argv[1:]
    taps = None
    if "--taps" in args:
        i = args.index("--taps")
        taps = int(args[i + 1])
        del args[i:i + 2]
    only = args or ["resnet50"]
    autotune.load_cache()
    dropped = [k for k in list(Fn._tuned) if isinstance(k, tuple) and k[0] in ("fwd", "dgb")
               and (taps is None or k[-1] == taps)]
    for k in dropped:
        del Fn._tuned[k]
    print(f"dropped {len(dropped)} fwd/dgb entries", flush=True)
    for name, b in CONFIGS:
        if name not in only:
            continue
        t0 = time.time()
        m = create_model(name, device="cuda", compute_dtype="bf16")
        n = autotune.tune_model(m, b, verbose=True, save=False)
        del m
        torch.cuda.empty_cache()
        print(f"{name} bs{b}: tuned {n} problems in {time.time() - t0:.0f} s", flush=True)
    autotune.save_cache()
    os.makedirs("gpurun_out", exist_ok=True)
    shutil.copy(autotune.DEFAULT_CACHE, "gpurun_out/mi355x.json")


if __name__ == "__main__":
    main()
