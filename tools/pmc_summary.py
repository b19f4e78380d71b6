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
            line = " ".join(f"{c}={v / disp:.4g}" for c, v in sorted(cs.items()))
            # derived: MFMA busy share of the busy time, LDS conflict share, L2 hit rate
            if "SQ_VALU_MFMA_BUSY_CYCLES" in cs and "GRBM_GUI_ACTIVE" in cs:
                # MFMA busy cycles are per SIMD-cycle summed over the chip: 1024 SIMDs
                line += f"  mfma_util={cs['SQ_VALU_MFMA_BUSY_CYCLES'] / (cs['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}"
            if "SQ_LDS_BANK_CONFLICT" in cs and cs.get("SQ_LDS_IDX_ACTIVE"):
                line += f"  lds_conflict={cs['SQ_LDS_BANK_CONFLICT'] / cs['SQ_LDS_IDX_ACTIVE']:.3f}"
            if "TCC_HIT_sum" in cs and (cs["TCC_HIT_sum"] + cs.get("TCC_MISS_sum", 0)) > 0:
                line += f"  l2_hit={cs['TCC_HIT_sum'] / (cs['TCC_HIT_sum'] + cs['TCC_MISS_sum']):.3f}"
            print(os.path.basename(d), k, line)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
