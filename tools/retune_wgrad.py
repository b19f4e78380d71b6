#!/usr/bin/env python3
"""Drop every weight-gradient entry of the in-tree autotune cache and re-tune them (after a
weight-grad kernel change) for the given model configs (default: all of tools/tune_all.py's);
forward / data-grad entries are kept."""
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
    only = sys.argv[1:]
    autotune.load_cache()
    dropped = [k for k in list(Fn._tuned) if str(k).startswith("wgrad") or (isinstance(k, tuple) and k[0] == "wgrad")]
    for k in dropped:
        del Fn._tuned[k]
    print(f"dropped {len(dropped)} wgrad entries", flush=True)
    for name, b in CONFIGS:
        if only and name not in only:
            continue
        t0 = time.time()
        m = create_model(name, device="cuda", compute_dtype="bf16")
        n = autotune.tune_model(m, b, verbose=True, save=True)
        del m
        torch.cuda.empty_cache()
        print(f"{name} bs{b}: tuned {n} problems in {time.time() - t0:.0f} s", flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    shutil.copy(autotune.DEFAULT_CACHE, "gpurun_out/mi355x.json")


if __name__ == "__main__":
    main()
