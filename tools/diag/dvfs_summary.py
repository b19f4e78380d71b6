"""Summarise a rocprofv3 --pmc GRBM_GUI_ACTIVE pass (tools/diag/dvfs_probe.sh): per conv kernel,
mean duration and effective clock = GRBM_GUI_ACTIVE / 8 XCDs / duration."""
import csv
import glob
import os
import sys

d, tag = sys.argv[1], sys.argv[2]
f = (glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True) or [None])[0]
if f is None:
    print(tag, "no counter csv under", d)
    sys.exit(0)
rows = list(csv.DictReader(open(f)))
by = {}
for r in rows:
    k = r.get("Kernel_Name", "")
    if "conv" not in k:
        continue
    name = r.get("Counter_Name")
    val = float(r.get("Counter_Value", 0))
    dur = (float(r.get("End_Timestamp", 0)) - float(r.get("Start_Timestamp", 0))) if r.get("End_Timestamp") else None
    by.setdefault(k[:70], []).append((name, val, dur, r.get("Dispatch_Id")))
for k, v in by.items():
    ga = [x for x in v if x[0] == "GRBM_GUI_ACTIVE"]
    durs = [x[2] for x in ga if x[2]]
    if not ga or not durs:
        print(tag, k, "n/a")
        continue
    tot_act = sum(x[1] for x in ga) / len(ga)
    dur = sum(durs) / len(durs)
    print(f"{tag}: {k} n={len(ga)} dur {dur / 1e3:.1f} us  GUI_ACTIVE {tot_act:.0f}  clock {tot_act / 8 / dur:.3f} GHz")
