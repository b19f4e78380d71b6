#!/usr/bin/env python3
"""tests/test_race_gpu.py's race detector pointed at the runtime's graph packet capture: the
data-parallel step (forked comm branches, 1-rank RCCL) with DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 in
the asynchronous arm vs the kernel-serialised reference (profiles/r2f_graph_packet_capture.txt)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_race_gpu import SCRIPT  # noqa: E402


ARGS = sys.argv[1:4]  # optional image size, batch (default 64 8), "tuned"


def run(extra, port):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
               LOCAL_WORLD_SIZE="1", **extra)
    out = subprocess.run([sys.executable, "-c", SCRIPT, ROOT, "dp", *ARGS], env=env, capture_output=True, text=True,
                         timeout=240)
    if out.returncode != 0:
        print(out.stderr[-2000:])
        sys.exit(out.returncode)
    return json.loads(out.stdout.strip().splitlines()[-1])


def main():
    ref = run({"AMD_SERIALIZE_KERNEL": "3", "AMD_SERIALIZE_COPY": "3", "HIP_LAUNCH_BLOCKING": "1"}, 29660)
    for pc in (os.environ.get("PC_SEQ") or "0 1 1 1 0").split():
        r = run({"DEBUG_CLR_GRAPH_PACKET_CAPTURE": pc}, 29661)
        same = r["losses"] == ref["losses"] and r["master"] == ref["master"]
        first = next((i for i, (a, b) in enumerate(zip(r["losses"], ref["losses"])) if a != b), None)
        print(f"DEBUG_CLR_GRAPH_PACKET_CAPTURE={pc}: {'bitwise equal to the serialised run' if same else 'DIFFERS'}"
              + ("" if same else f" (first differing step: {first})"), flush=True)


if __name__ == "__main__":
    main()
