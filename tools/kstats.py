#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--stats`` kernel table (``*_kernel_stats.csv``) per training step,
grouped by kernel class. Usage: python tools/kstats.py gpurun_out/prof/run_kernel_stats.csv --steps 13"""
import argparse
import csv
import re

CLASSES = [("conv fwd/dgrad (igemm)", r"conv_igemm|conv_p3_persist|conv3x3"), ("conv wgrad", r"wgrad"), ("stem", r"stem"),
           ("BN fwd apply", r"bn_apply|bn_relu_maxpool"), ("BN bwd", r"bn_bwd"), ("pool", r"pool|gap_"),
           ("optimizer / pack", r"sgd|weight_pack|nonfinite"), ("torch fills / misc", r"at::|at6native|rocclr"),
           ("loss / fc", r"softmax|colsum")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=float, default=13.0)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {a.csv}: {sum(int(r['Calls']) for r in rows)} dispatches, {tot / 1e6:.2f} ms GPU kernel time, "
          f"{tot / 1e6 / a.steps:.3f} ms per step over {a.steps:g} steps")
    print(f"{'kernel':100s} {'calls':>6s} {'ms/step':>8s} {'avg_us':>8s} {'%':>6s}")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:a.top]:
        t = float(r["TotalDurationNs"])
        print(f"{r['Name'][:100]:100s} {int(r['Calls']):6d} {t / 1e6 / a.steps:8.3f} {float(r['AverageNs']) / 1e3:8.1f} "
              f"{100 * t / tot:6.2f}")
    print("\n# per class (ms/step)")
    seen = set()
    for cname, pat in CLASSES:
        t = sum(float(r["TotalDurationNs"]) for r in rows if re.search(pat, r["Name"]) and r["Name"] not in seen)
        seen |= {r["Name"] for r in rows if re.search(pat, r["Name"])}
        print(f"{cname:30s} {t / 1e6 / a.steps:8.3f}")
    rest = sum(float(r["TotalDurationNs"]) for r in rows if r["Name"] not in seen)
    print(f"{'other':30s} {rest / 1e6 / a.steps:8.3f}")


if __name__ == "__main__":
    main()
