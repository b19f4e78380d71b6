#!/usr/bin/env python3
"""Per-step row-loss hashes of the race detector's deterministic single-graph run (tests/test_race_gpu.py
SCRIPT, 64 px, batch 8) under {packet capture on, off} x {async, serialised}, twice each: which
runs agree bit for bit."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_race_gpu as R  # noqa: E402

os.environ["RACE_STEPS"] = "6"
os.environ["RACE_SWITCHES"] = sys.argv[1] if len(sys.argv) > 1 else ""
for pc in ("1", "0"):
    os.environ["DEBUG_CLR_GRAPH_PACKET_CAPTURE"] = pc
    for ser in (False, True, False):
        r = R._run("single", serialize=ser)
        print(json.dumps({"pc": pc, "serialised": ser, "switches": os.environ["RACE_SWITCHES"],
                          "steps": [h[:8] for h in r["losses"]], "master": r["master"][:8]}), flush=True)
