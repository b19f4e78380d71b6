#!/usr/bin/env python3
"""Every fp32 ResNet-50 plane-GEMM problem at its tuned plan: isolated time (autotune._time), launches
per step, x6-MFMA efficiency and the step share -- where the GEMM time goes, problem by problem.

    python tools/diag/fp32_problem_table.py [--batch 64]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from azure_hc_intel_tf_amd.models import create_model  # noqa: E402
from azure_hc_intel_tf_amd.ops import autotune  # noqa: E402
from azure_hc_intel_tf_amd.ops import functional as Fn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--dtype", default="fp32", help="fp32 (plane GEMMs) or bf16")
    a = ap.parse_args()
    m = create_model("resnet50", device="cuda", compute_dtype=a.dtype)
    autotune.load_cache()
    m.ps.repack()
    probs = autotune.model_problems(m, a.batch)
    rows = []
    for k, (cnt, cands, run) in probs.items():
        cur = Fn._tuned.get(k)
        t = autotune._time(lambda: run(cur)) * 1000
        if k[0] in ("wgrad3", "wgrad"):
            _, nout, kk, mm, taps = k
            fl = 2.0 * nout * kk * mm
        else:
            _, mm, n, kk, taps = k
            fl = 2.0 * mm * n * kk
        rows.append((cnt * t, k, cnt, cur, t, fl / t / 1e6))
    rows.sort(key=lambda r: -r[0])
    tot = sum(r[0] for r in rows)
    print(f"# {len(rows)} problems, isolated sum x launches = {tot / 1000:.3f} ms/step")
    for tt, k, cnt, cur, t, tf in rows:
        x = 6 if a.dtype == "fp32" else 1
        print(f"{str(k):44s} x{cnt:2d} plan {str(cur):10s} {t:7.1f} us  {tf:5.0f} TF  MFMA {x * tf / 25:4.0f}%  "
              f"step {tt / 1000:.3f} ms ({100 * tt / tot:4.1f}%)", flush=True)


if __name__ == "__main__":
    main()
