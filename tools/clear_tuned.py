#!/usr/bin/env python3
"""Drop tuning-table entries by key prefix so the next run re-tunes them:
python tools/clear_tuned.py fwd3 wgrad3"""
import json
import os
import sys

P = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "azure_hc_intel_tf_amd", "tuned",
                 "mi355x.json")
d = json.load(open(P))
pre = tuple(a + "|" for a in sys.argv[1:])
n0 = len(d["entries"])
d["entries"] = {k: v for k, v in d["entries"].items() if not k.startswith(pre)}
json.dump(d, open(P, "w"), indent=0, sort_keys=True)
print(f"dropped {n0 - len(d['entries'])} entries")
