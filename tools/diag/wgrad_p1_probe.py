#!/usr/bin/env python3
"""16-bit weight gradient: the plane kernel's one-plane form (wgrad cfg 15-22, conv_p3_wgrad.h NP=1)
against the tuned plan of every bf16 ResNet-50 weight-gradient problem (autotune._time, isolated
step-like launches). With --retune the problems of this model whose best new plan wins by > 3% are
re-tuned over ALL candidates and the in-tree table saved (other models' entries untouched).

    python tools/diag/wgrad_p1_probe.py [--batch 64] [--retune]
"""
import argparse
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from azure_hc_intel_tf_amd.models import create_model  # noqa: E402
from azure_hc_intel_tf_amd.ops import autotune  # noqa: E402
from azure_hc_intel_tf_amd.ops import functional as Fn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--retune", action="store_true")
    a = ap.parse_args()
    m = create_model("resnet50", device="cuda", compute_dtype="bf16")
    autotune.load_cache()
    m.ps.repack()
    probs = autotune.model_problems(m, a.batch)
    tot_cur = tot_new = 0.0
    changed = 0
    for k, (cnt, cands, run) in probs.items():
        if k[0] != "wgrad":
            continue
        cur = Fn._tuned.get(k)
        cur = tuple(cur) if cur is not None else None
        t_cur = autotune._time(lambda: run(cur)) * 1000
        new = [c for c in cands if c[0] >= 15]
        tn = {c: autotune._time(lambda: run(c)) * 1000 for c in new}
        bn = min(tn, key=tn.get)
        best_t = min(t_cur, tn[bn])
        tot_cur += cnt * t_cur
        tot_new += cnt * best_t
        print(f"{k} x{cnt}: tuned {cur} {t_cur:.1f} us | best one-plane {bn} {tn[bn]:.1f} us "
              f"({100 * (t_cur - tn[bn]) / t_cur:+.0f}%)", flush=True)
        if a.retune and tn[bn] < 0.97 * t_cur:
            Fn._tuned[k] = list(bn)
            changed += 1
    print(f"# per step (x count): tuned {tot_cur / 1000:.3f} ms, with the one-plane cfgs where faster "
          f"{tot_new / 1000:.3f} ms", flush=True)
    if a.retune:
        autotune.save_cache()
        os.makedirs("gpurun_out", exist_ok=True)
        shutil.copy(autotune.DEFAULT_CACHE, "gpurun_out/mi355x.json")
        print(f"# {changed} entries changed; table saved", flush=True)


if __name__ == "__main__":
    main()
