"""Checkpoint / resume (tf_cnn_benchmarks ``--train_dir`` / ``--save_model_steps`` /
``--save_model_secs`` role; SURVEY.md §5 "Checkpoint / resume").

Rank 0 writes ``model.ckpt-<step>.pt`` holding the flat fp32 masters, momentum slots, BN
moving statistics and the variable-name table; files contain tensors + plain Python
containers only and are loaded with ``torch.load(weights_only=True)``. Resume: rank 0
restores the latest checkpoint, then ``hvd.broadcast_global_variables(0)`` syncs every
worker. Writes are atomic (tmp file + rename)."""
from __future__ import annotations

import glob
import os
import re
from typing import Optional

import torch

_PAT = re.compile(r"model\.ckpt-(\d+)\.pt$")


def save(train_dir: str, step: int, ps, keep: int = 5) -> str:
    os.makedirs(train_dir, exist_ok=True)
    sd = ps.state_dict()
    sd["global_step"] = int(step)
    path = os.path.join(train_dir, f"model.ckpt-{int(step)}.pt")
    tmp = path + ".tmp"
    torch.save(sd, tmp)
    os.replace(tmp, path)
    with open(os.path.join(train_dir, "checkpoint"), "w") as f:
        f.write(f'model_checkpoint_path: "{os.path.basename(path)}"\n')
    for old in list_checkpoints(train_dir)[:-keep]:
        try:
            os.remove(old[1])
        except OSError:
            pass
    return path


def list_checkpoints(train_dir: str):
    out = []
    for p in glob.glob(os.path.join(train_dir, "model.ckpt-*.pt")):
        m = _PAT.search(p)
        if m:
            out.append((int(m.group(1)), p))
    return sorted(out)


def latest(train_dir: str) -> Optional[str]:
    c = list_checkpoints(train_dir) if os.path.isdir(train_dir) else []
    return c[-1][1] if c else None


def restore_latest(train_dir: str, ps) -> int:
    """Load the newest checkpoint into ``ps``; returns its global step (0 if none)."""
    path = latest(train_dir)
    if path is None:
        return 0
    sd = torch.load(path, map_location="cpu", weights_only=True)
    ps.load_state_dict(sd)
    return int(sd.get("global_step", 0))
