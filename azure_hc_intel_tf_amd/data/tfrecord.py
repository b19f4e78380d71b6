"""TFRecord / tf.train.Example I/O through the native ``_hcb_data`` library.

The reference's real-data runs read ImageNet TFRecord shards (``--data_dir=... --data_name=
imagenet``, /root/reference/benchmark-scripts/run-tf-sing-ucx-openmpi.sh:19,80-81; 20 of the
1024 train shards). TensorFlow is not part of this engine, so the record framing (masked
CRC-32C), the Example wire format and the ImageNet feature keys are implemented natively in
``csrc/data/tfrecord.cpp``; this module is the Python face of it plus an ImageNet-style
Example builder used by the tests and ``tools/make_fake_imagenet.py``.
"""
from __future__ import annotations

import glob
import importlib
import os
import sys
from typing import Dict, Iterator, List, Optional, Sequence

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_MOD = None


def native():
    """The ``_hcb_data`` extension (built in-tree by ``_build.build_data`` if missing)."""
    global _MOD
    if _MOD is not None:
        return _MOD
    # HCB_DATA_LIB_DIR: load another build of the library (e.g. the ASan/UBSan build of
    # tools/sanitize_data.sh) instead of the in-tree one
    d = os.environ.get("HCB_DATA_LIB_DIR") or _PKG
    if d not in sys.path:
        sys.path.insert(0, d)
    try:
        _MOD = importlib.import_module("_hcb_data")
    except ImportError:
        from .. import _build

        _build.build_data()
        importlib.invalidate_caches()
        _MOD = importlib.import_module("_hcb_data")
    return _MOD


def write_records(path: str, records: Sequence[bytes]) -> None:
    w = native().RecordWriter(path)
    for r in records:
        w.write(r)
    w.close()


def read_records(path: str, verify_crc: bool = True) -> Iterator[bytes]:
    r = native().RecordReader(path, verify_crc)
    while True:
        rec = r.next()
        if rec is None:
            return
        yield rec


def parse_example(rec: bytes) -> Dict[str, list]:
    return native().parse_example(rec)


def encode_example(features: Dict[str, object]) -> bytes:
    """features: name -> bytes / str / int / float or a list of one kind."""
    return native().encode_example(features)


def imagenet_example(jpeg: bytes, label: int, height: int, width: int, synset: str = "n00000000",
                     boxes: Optional[List[Sequence[float]]] = None, filename: str = "") -> bytes:
    """An Example with the feature keys of the standard ImageNet TFRecord build
    (image/encoded, image/class/label, image/height, image/width, image/object/bbox/*)."""
    boxes = boxes or []
    return encode_example({
        "image/encoded": [jpeg],
        "image/format": [b"JPEG"],
        "image/class/label": [int(label)],
        "image/class/synset": [synset.encode()],
        "image/height": [int(height)],
        "image/width": [int(width)],
        "image/channels": [3],
        "image/colorspace": [b"RGB"],
        "image/filename": [filename.encode()],
        "image/object/bbox/ymin": [float(b[0]) for b in boxes],
        "image/object/bbox/xmin": [float(b[1]) for b in boxes],
        "image/object/bbox/ymax": [float(b[2]) for b in boxes],
        "image/object/bbox/xmax": [float(b[3]) for b in boxes],
        "image/object/bbox/label": [int(label)] * len(boxes),
    })


def find_shards(data_dir: str, subset: str = "train") -> List[str]:
    """tf_cnn_benchmarks' ImageNet file pattern: ``<data_dir>/<subset>-*-of-*``."""
    files = sorted(glob.glob(os.path.join(data_dir, f"{subset}-*-of-*")))
    if not files:
        raise FileNotFoundError(f"no {subset}-*-of-* TFRecord shards in {data_dir}")
    return files
