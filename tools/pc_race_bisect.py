#!/usr/bin/env python3
"""Graph packet capture (DEBUG_CLR_GRAPH_PACKET_CAPTURE=1) bisection on the race detector of
tests/test_race_gpu.py: the deterministic single-graph ResNet-50 run (64 px, batch 8) async vs
serialised, with module switches flipped one at a time (RACE_SWITCHES). One line per run:
variant, equal / DIFFER (first differing step)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_race_gpu as R  # noqa: E402

VARIANTS = [("baseline", ""), ("baseline", ""), ("no fused BN backward", "L.FUSE_BN_BWD=0"),
            ("no fused stem pool", "L.FUSE_STEM_POOL=0"), ("no fused shortcut BN", "L.FUSE_RES_BN=0"),
            ("no stem s2d", "L.STEM_S2D=0"), ("no BN shift", "L.BN_SHIFT=0"), ("no dgrad phases", "Fn.DGRAD_PHASES=0")]


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "single"
    os.environ["RACE_STEPS"] = os.environ.get("RACE_STEPS", "6")
    for label, sw in VARIANTS:
        os.environ["RACE_SWITCHES"] = sw
        a = R._run(mode, serialize=False)
        s = R._run(mode, serialize=True)
        diff = [i for i, (x, y) in enumerate(zip(a["losses"], s["losses"])) if x != y]
        print(json.dumps({"variant": label, "switches": sw, "mode": mode, "equal": not diff and a["master"] == s["master"],
                          "first_diff_step": diff[0] if diff else None,
                          "pc": os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE")}), flush=True)


if __name__ == "__main__":
    main()
