#!/usr/bin/env python3
"""Per-dispatch comparison of two rocprofv3 kernel traces of the same training step (e.g. two tuned
tables, or two kernel builds): the last STEPS graph replays of each trace are split into steps at the
step's first kernel, dispatch i of one step is matched with dispatch i of the other (same model, same
launch order), and the per-position median durations are compared.

    python tools/trace_diff.py A/run_kernel_trace.csv B/run_kernel_trace.csv [--steps 8] [--top 25]
"""
import argparse
import csv
import statistics


def steps_of(path, nsteps, marker):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    if len(starts) < nsteps + 1:
        raise SystemExit(f"{path}: only {len(starts)} step markers ({marker!r})")
    out = []
    for a, b in zip(starts[-nsteps - 1:-1], starts[-nsteps:]):
        out.append([(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
                    for r in rows[a:b]])
    return out


def short(name, n=70):
    name = name.replace("hcb::", "").replace("(hcb::ConvParams)", "").replace("(hcb::WgradParams)", "")
    return name[:n]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--marker", default="zero_bufs_kernel", help="the step's first kernel")
    a = ap.parse_args()
    sa, sb = steps_of(a.a, a.steps, a.marker), steps_of(a.b, a.steps, a.marker)
    na, nb = len(sa[0]), len(sb[0])
    print(f"# dispatches per step: A {na}, B {nb}")
    if na != nb:
        print("# different launch sequences: per-position comparison not meaningful")
    n = min(na, nb)
    rows = []
    for i in range(n):
        ta = statistics.median(s[i][1] for s in sa)
        tb = statistics.median(s[i][1] for s in sb)
        rows.append((tb - ta, i, ta, tb, sa[0][i][0], sb[0][i][0]))
    tot_a = sum(r[2] for r in rows)
    tot_b = sum(r[3] for r in rows)
    print(f"# sum of per-dispatch medians: A {tot_a / 1000:.3f} ms, B {tot_b / 1000:.3f} ms ({tot_b - tot_a:+.1f} us)")
    print("# largest B - A differences (us): position, A us, B us, A kernel | B kernel")
    for d, i, ta, tb, ka, kb in sorted(rows, key=lambda r: -abs(r[0]))[:a.top]:
        same = "" if ka == kb else f" | {short(kb)}"
        print(f"{d:+8.1f}  #{i:3d}  {ta:8.1f} {tb:8.1f}  {short(ka)}{same}")


if __name__ == "__main__":
    main()
