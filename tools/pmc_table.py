#!/usr/bin/env python3
"""Per-kernel summary of one rocprofv3 --pmc run (run_counter_collection.csv): counters per dispatch
and the derived shares -- MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs x the dispatch's
GRBM_GUI_ACTIVE / 8 XCDs), wave-cycle split into waiting (s_waitcnt / barrier), issue-stalled and
issuing (SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY, quad-cycles, of SQ_WAVE_CYCLES), LDS
bank-conflict share. python tools/pmc_table.py gpurun_out/<run>_pmc [name-filter]"""
import collections
import csv
import glob
import os
import sys


def main(root, filt=""):
    files = glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in files:
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "?")
            if filt and filt not in k:
                continue
            agg[k][row["Counter_Name"]] += float(row["Counter_Value"])
            disp[k].add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
    rows = []
    for k, cs in agg.items():
        n = max(len(disp[k]), 1)
        g = cs.get("GRBM_GUI_ACTIVE", 0.0)
        mf = cs.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        wc = cs.get("SQ_WAVE_CYCLES", 0.0)
        d = {"calls": n, "grbm_per_call": g / n}
        if g:
            d["mfma_util"] = mf / (g / 8 * 1024)
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in cs:
                    d[c.replace("SQ_", "").lower()] = cs[c] / wc
        if cs.get("TCC_HIT_sum") or cs.get("TCC_MISS_sum"):
            h, mi = cs.get("TCC_HIT_sum", 0.0), cs.get("TCC_MISS_sum", 0.0)
            d["l2_hit"] = h / max(h + mi, 1.0)
            d["l2_req_per_call"] = (h + mi) / n
        if cs.get("TCP_TCC_READ_REQ_sum"):
            d["l1_l2_rd_req_per_call"] = cs["TCP_TCC_READ_REQ_sum"] / n
        if cs.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_conflict"] = cs.get("SQ_LDS_BANK_CONFLICT", 0.0) / cs["SQ_LDS_IDX_ACTIVE"]
        rows.append((g, k, d))
    rows.sort(reverse=True)
    for g, k, d in rows[:40]:
        print(f"{k[:90]:90s} " + " ".join(f"{a}={v:.3g}" for a, v in d.items()))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc", sys.argv[2] if len(sys.argv) > 2 else "")
