#!/usr/bin/env python3
"""The race detector of tests/test_race_gpu.py at the benchmark's size (224 px, batch 64, the
autotuned kernel configs -- incl. the 3x3 patch kernels): the single-graph step and the
data-parallel overlap step (1-rank RCCL) each run asynchronously and fully kernel-serialised
(AMD_SERIALIZE_KERNEL=3 AMD_SERIALIZE_COPY=3 HIP_LAUNCH_BLOCKING=1), deterministic mode; the
per-row losses and the final weights must be bitwise equal."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_race_gpu import SCRIPT  # noqa: E402


def run(mode, serialize, port):
    env = dict(os.environ, RACE_STEPS=os.environ.get("RACE_STEPS", "6"))
    if serialize:
        env.update(AMD_SERIALIZE_KERNEL="3", AMD_SERIALIZE_COPY="3", HIP_LAUNCH_BLOCKING="1")
    if mode == "dp":
        env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
                   LOCAL_WORLD_SIZE="1")
    out = subprocess.run([sys.executable, "-c", SCRIPT, ROOT, mode, "224", "64", "tuned"], env=env,
                         capture_output=True, text=True, timeout=500)
    if out.returncode != 0:
        print(out.stderr[-2000:])
        sys.exit(1)
    return json.loads(out.stdout.strip().splitlines()[-1])


def main():
    ok = True
    dts = os.environ.get("RACE_DTYPES", "bf16,fp32").split(",")  # fp32: the headline precision
    for j, dt in enumerate(dts):
        os.environ["RACE_DTYPE"] = dt
        for i, mode in enumerate(("single", "dp")):
            a = run(mode, False, 29670 + 4 * j + 2 * i)
            s = run(mode, True, 29671 + 4 * j + 2 * i)
            same = a["losses"] == s["losses"] and a["master"] == s["master"]
            ok &= same
            print(json.dumps({"mode": mode, "dtype": dt, "size": 224, "batch": 64, "tuned": True,
                              "overlap": a["overlap"], "bitwise_equal": same}), flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
