#!/usr/bin/env python3
"""Write a small ImageNet-format TFRecord dataset (random JPEGs, labels in [1, 1000], one
labelled box each) for exercising the ``--data_dir`` path without the real dataset:

    python tools/make_fake_imagenet.py /tmp/fake_imagenet --shards 4 --per_shard 64

Files are named like the standard build (``train-00000-of-00004``, ``validation-...``).
"""
import argparse
import io
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from azure_hc_intel_tf_amd.data.tfrecord import imagenet_example, write_records  # noqa: E402


def fake_jpeg(rng, h, w, quality=85):
    from PIL import Image

    base = rng.integers(0, 256, size=(max(h // 8, 1), max(w // 8, 1), 3), dtype=np.uint8)
    img = Image.fromarray(base).resize((w, h), Image.BILINEAR)
    b = io.BytesIO()
    img.save(b, format="JPEG", quality=quality)
    return b.getvalue()


def make(out_dir, shards=4, per_shard=64, subset="train", seed=0, min_side=160, max_side=500):
    os.makedirs(out_dir, exist_ok=True)
    rng = np.random.default_rng(seed)
    paths = []
    for s in range(shards):
        recs = []
        for i in range(per_shard):
            h, w = (int(v) for v in rng.integers(min_side, max_side + 1, size=2))
            y0, x0 = rng.uniform(0, 0.4, size=2)
            y1, x1 = rng.uniform(0.6, 1.0, size=2)
            label = int(rng.integers(1, 1001))
            recs.append(imagenet_example(fake_jpeg(rng, h, w), label, h, w, boxes=[(y0, x0, y1, x1)],
                                         filename=f"{subset}_{s}_{i}.JPEG"))
        p = os.path.join(out_dir, f"{subset}-{s:05d}-of-{shards:05d}")
        write_records(p, recs)
        paths.append(p)
    return paths


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("out_dir")
    ap.add_argument("--shards", type=int, default=4)
    ap.add_argument("--per_shard", type=int, default=64)
    ap.add_argument("--subset", default="train")
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    for p in make(a.out_dir, a.shards, a.per_shard, a.subset, a.seed):
        print(p)
