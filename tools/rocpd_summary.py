#!/usr/bin/env python3
"""Summarise a rocprofv3 (ROCm 7.2) ``*_results.db`` kernel trace: per-kernel totals and the
dispatch sequence of one training step. Usage:

    python tools/rocpd_summary.py gpurun_out/prof/run_results.db [--steps N] [--seq]
"""
import argparse
import collections
import glob
import os
import sqlite3
import sys


def load(db):
    con = sqlite3.connect(db)
    cur = con.cursor()
    q = ("select d.start, d.end, s.kernel_name, d.grid_size_x, d.grid_size_y, d.workgroup_size_x, "
         "s.arch_vgpr_count, s.accum_vgpr_count, s.group_segment_size, d.group_segment_size "
         "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start")
    return list(cur.execute(q))


def short(name, n=90):
    name = name.replace("void ", "")
    if "(" in name:
        name = name[:name.index("(")] if not name.startswith("hcb::") else name
    return name[:n]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db", nargs="?", default=None)
    ap.add_argument("--steps", type=int, default=10, help="timed steps in the profiled run (for per-step numbers)")
    ap.add_argument("--seq", action="store_true", help="print the dispatch sequence of the last step")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    db = a.db or sorted(glob.glob("gpurun_out/prof/**/*results.db", recursive=True))[-1]
    rows = load(db)
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    for st, en, name, gx, gy, wx, vg, ag, lds, dlds in rows:
        k = short(name, 160)
        tot[k] += (en - st) / 1e3
        cnt[k] += 1
    all_us = sum(tot.values())
    print(f"# {db}: {len(rows)} dispatches, {all_us / 1e3:.2f} ms total GPU kernel time")
    print(f"{'kernel':100s} {'calls':>7s} {'total_ms':>9s} {'avg_us':>8s} {'%':>6s}")
    for k, v in sorted(tot.items(), key=lambda x: -x[1])[:a.top]:
        print(f"{k[:100]:100s} {cnt[k]:7d} {v / 1e3:9.3f} {v / cnt[k]:8.1f} {100 * v / all_us:6.2f}")
    if a.seq:
        # last step = dispatches after the last sgd_momentum but one
        idx = [i for i, r in enumerate(rows) if "sgd_momentum" in r[2]]
        if len(idx) >= 2:
            seg = rows[idx[-2] + 1: idx[-1] + 1]
            print(f"\n# dispatch sequence of the last step ({len(seg)} kernels, "
                  f"{(seg[-1][1] - seg[0][0]) / 1e6:.3f} ms wall, {sum(r[1] - r[0] for r in seg) / 1e6:.3f} ms busy)")
            for st, en, name, gx, gy, wx, vg, ag, lds, dlds in seg:
                print(f"{(en - st) / 1e3:9.1f} us  grid={gx // max(wx, 1)}x{gy} vgpr={vg}+{ag} lds={dlds}  {short(name, 110)}")


if __name__ == "__main__":
    main()
