#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counter CSVs per kernel: python tools/pmc_summary.py gpurun_out/pmc"""
import collections
import csv
import glob
import os
import sys


def main(root):
    for d in sorted(glob.glob(os.path.join(root, "*.*"))):
        if not os.path.isdir(d):
            continue
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        n = collections.Counter()
        for f in files:
            for row in csv.DictReader(open(f)):
                k = row.get("Kernel_Name", "?")[:60]
                agg[k][row["Counter_Name"]] += float(row["Counter_Value"])
                n[(k, row["Counter_Name"])] += 1
        for k, cs in agg.items():
            if "conv" not in k:
                continue
            disp = max(n[(k, c)] for c in cs)
            print(os.path.basename(d), k, " ".join(f"{c}={v / disp:.3g}" for c, v in sorted(cs.items())))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
