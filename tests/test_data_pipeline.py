"""Real-data input pipeline (``--data_dir``): native TFRecord / tf.Example / crop-window /
prefetch core and the preprocessing reference (CPU), plus an end-to-end CPU run of the
tf_cnn_benchmarks CLI on a small ImageNet-format dataset written by
tools/make_fake_imagenet.py. No real ImageNet (and no TensorFlow) exists here: wire-format
parity is pinned against the protobuf runtime with a dynamically built tf.train.Example
descriptor and the CRC against the published CRC-32C check value."""
import io
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from azure_hc_intel_tf_amd.data import tfrecord as T  # noqa: E402
from azure_hc_intel_tf_amd.data.imagenet import decode_crop, preprocess_reference  # noqa: E402


@pytest.fixture(scope="module")
def fake_dir(tmp_path_factory):
    import make_fake_imagenet

    d = tmp_path_factory.mktemp("fake_imagenet")
    make_fake_imagenet.make(str(d), shards=3, per_shard=12, subset="train", seed=1)
    make_fake_imagenet.make(str(d), shards=1, per_shard=8, subset="validation", seed=2)
    return str(d)


def test_crc32c_check_value_and_mask():
    n = T.native()
    assert n.crc32c(b"123456789") == 0xE3069283
    c = n.crc32c(b"hello tfrecord")
    assert n.masked_crc32c(b"hello tfrecord") == ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF
    long = bytes(range(256)) * 37 + b"xyz"  # exercises the 8-byte loop and the tail
    assert n.crc32c(long) == _crc32c_bitwise(long)


def _crc32c_bitwise(data):
    crc = 0xFFFFFFFF
    for b in data:
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ (0x82F63B78 if crc & 1 else 0)
    return crc ^ 0xFFFFFFFF


def _example_class():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    f = descriptor_pb2.FileDescriptorProto(name="hcb_example_test.proto", package="hcbtest", syntax="proto3")
    R, O = descriptor_pb2.FieldDescriptorProto.LABEL_REPEATED, descriptor_pb2.FieldDescriptorProto.LABEL_OPTIONAL
    Ty = descriptor_pb2.FieldDescriptorProto
    for name, t in (("BytesList", Ty.TYPE_BYTES), ("FloatList", Ty.TYPE_FLOAT), ("Int64List", Ty.TYPE_INT64)):
        m = f.message_type.add(name=name)
        m.field.add(name="value", number=1, label=R, type=t)
    feat = f.message_type.add(name="Feature")
    feat.oneof_decl.add(name="kind")
    for i, (n, tn) in enumerate((("bytes_list", "BytesList"), ("float_list", "FloatList"),
                                 ("int64_list", "Int64List"))):
        feat.field.add(name=n, number=i + 1, label=O, type=Ty.TYPE_MESSAGE, type_name=".hcbtest." + tn,
                       oneof_index=0)
    fs = f.message_type.add(name="Features")
    entry = fs.nested_type.add(name="FeatureEntry")
    entry.options.map_entry = True
    entry.field.add(name="key", number=1, label=O, type=Ty.TYPE_STRING)
    entry.field.add(name="value", number=2, label=O, type=Ty.TYPE_MESSAGE, type_name=".hcbtest.Feature")
    fs.field.add(name="feature", number=1, label=R, type=Ty.TYPE_MESSAGE, type_name=".hcbtest.Features.FeatureEntry")
    ex = f.message_type.add(name="Example")
    ex.field.add(name="features", number=1, label=O, type=Ty.TYPE_MESSAGE, type_name=".hcbtest.Features")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(f)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("hcbtest.Example"))


def test_example_wire_format_matches_protobuf_runtime():
    Example = _example_class()
    feats = {"image/encoded": [b"\xff\xd8jpegbytes\x00\x01"], "image/class/label": [417],
             "image/object/bbox/xmin": [0.25, 0.5], "big": [2 ** 40, -3], "empty": []}
    ours = T.encode_example(feats)
    msg = Example()
    msg.ParseFromString(ours)  # the protobuf runtime reads what we wrote
    fm = msg.features.feature
    assert list(fm["image/encoded"].bytes_list.value) == [b"\xff\xd8jpegbytes\x00\x01"]
    assert list(fm["image/class/label"].int64_list.value) == [417]
    assert np.allclose(list(fm["image/object/bbox/xmin"].float_list.value), [0.25, 0.5])
    assert list(fm["big"].int64_list.value) == [2 ** 40, -3]
    # and we read what the protobuf runtime writes
    m2 = Example()
    m2.features.feature["a"].bytes_list.value.extend([b"x", b"yz"])
    m2.features.feature["b"].float_list.value.extend([1.5, -2.0])
    m2.features.feature["c"].int64_list.value.extend([7, 2 ** 33])
    back = T.parse_example(m2.SerializeToString())
    assert back["a"] == [b"x", b"yz"] and back["b"] == [1.5, -2.0] and back["c"] == [7, 2 ** 33]


def test_tfrecord_roundtrip_and_corruption(tmp_path):
    p = str(tmp_path / "x.tfrecord")
    recs = [b"", b"a", os.urandom(100000), b"last"]
    T.write_records(p, recs)
    assert list(T.read_records(p)) == recs
    raw = bytearray(open(p, "rb").read())
    raw[len(raw) - 6] ^= 0x01  # a payload byte of the last record
    open(p, "wb").write(bytes(raw))
    with pytest.raises(RuntimeError, match="CRC"):
        list(T.read_records(p))
    assert len(list(T.read_records(p, verify_crc=False))) == 4


def test_jpeg_dims_and_decode_crop():
    from PIL import Image

    import make_fake_imagenet

    rng = np.random.default_rng(0)
    jpeg = make_fake_imagenet.fake_jpeg(rng, 333, 457)
    assert T.native().jpeg_dims(jpeg) == (333, 457, 3)
    assert T.native().jpeg_dims(b"not a jpeg") is None
    full = np.asarray(Image.open(io.BytesIO(jpeg)).convert("RGB"))
    c = decode_crop(jpeg, (10, 20, 100, 150), (333, 457), 224, 4 * 224)
    assert c.shape == (100, 150, 3) and np.array_equal(c, full[10:110, 20:170])
    # DCT-domain downscale kicks in when the crop is >= 2x the output on both sides
    c2 = decode_crop(jpeg, (0, 0, 333, 457), (333, 457), 64, 4 * 64)
    assert c2.shape[0] < 333 and min(c2.shape[:2]) >= 64


def test_distorted_crop_semantics():
    n = T.native()
    H, W = 300, 400
    seen = set()
    for seed in range(200):
        y, x, h, w = n.distorted_crop(H, W, [(0.2, 0.2, 0.8, 0.8)], seed=seed)
        assert 0 <= y and 0 <= x and y + h <= H and x + w <= W and h > 0 and w > 0
        if (h, w) != (H, W):
            assert 0.05 * H * W - 1e-6 <= h * w <= H * W
            assert 0.75 - 0.02 <= w / h <= 1.33 + 0.02
            # min_object_covered = 0.1 of the labelled box
            iy = max(0, min(0.8 * H, y + h) - max(0.2 * H, y))
            ix = max(0, min(0.8 * W, x + w) - max(0.2 * W, x))
            assert iy * ix >= 0.1 * (0.6 * H) * (0.6 * W) - 1e-3
        seen.add((y, x, h, w))
    assert len(seen) > 150  # random
    assert n.distorted_crop(H, W, [], seed=5) == n.distorted_crop(H, W, [], seed=5)  # deterministic
    assert n.central_crop(H, W, 0.875) == ((H - 262) // 2, (W - 350) // 2, 262, 350)


def test_prefetcher_shards_ranks_and_epochs(fake_dir):
    files = T.find_shards(fake_dir, "train")
    assert len(files) == 3
    n = T.native()
    labels = {}
    for rank in range(2):
        pf = n.Prefetcher(files, rank=rank, world=2, threads=2, shuffle_buffer=4, seed=3, train=False, loop=False)
        got = pf.next(1000)
        pf.stop()
        labels[rank] = [s[1] for s in got]
        assert all(s[3] == 0 for s in got)  # eval: no flips
    # file i -> rank i % 2: rank 0 reads shards 0, 2; rank 1 reads shard 1
    assert len(labels[0]) == 24 and len(labels[1]) == 12
    alls = [T.parse_example(r) for f in files for r in T.read_records(f)]
    assert sorted(labels[0] + labels[1]) == sorted(e["image/class/label"][0] for e in alls)
    # looping + shuffling: more than one epoch is served, crops are inside the image
    pf = n.Prefetcher(files[:1], threads=1, shuffle_buffer=8, seed=4, train=True, loop=True)
    got = pf.next(30)
    assert pf.epochs >= 2 and len(got) == 30
    for jpeg, lab, (y, x, h, w), flip, (H, W) in got:
        assert 0 <= y and y + h <= H and 0 <= x and x + w <= W and flip in (0, 1)
    pf.stop()


def test_preprocess_reference_exact_on_identity_size():
    rng = np.random.default_rng(1)
    crop = rng.integers(0, 256, size=(16, 16, 3), dtype=np.uint8)
    out = torch.empty(2, 16, 16, 8, dtype=torch.float32)
    preprocess_reference([crop, crop], [0, 1], out)
    ref = torch.from_numpy(crop).float() / 127.5 - 1.0
    assert torch.allclose(out[0, :, :, :3], ref, atol=1e-6)
    assert torch.allclose(out[1, :, :, :3], ref.flip(1), atol=1e-6)
    assert out[..., 3:].abs().max() == 0
    # downscale by 2 samples every other source pixel (TF1 legacy: src = dst * in / out)
    big = rng.integers(0, 256, size=(32, 32, 3), dtype=np.uint8)
    o2 = torch.empty(1, 16, 16, 3)
    preprocess_reference([big], [0], o2)
    assert torch.allclose(o2[0], torch.from_numpy(big[::2, ::2].copy()).float() / 127.5 - 1.0, atol=1e-6)


def test_imagenet_loader_cpu(fake_dir):
    from azure_hc_intel_tf_amd.data.imagenet import ImageNetLoader

    ld = ImageNetLoader(fake_dir, 4, 32, 3, "cpu", train=True, seed=0, reader_threads=2, decode_threads=2, depth=2)
    img = torch.zeros(4, 32, 32, 3)
    lab = torch.zeros(4, dtype=torch.int64)
    seen = []
    for _ in range(5):
        ld.next_into(img, lab)
        assert img.abs().max() <= 1.0 + 1e-6 and img.std() > 0.01
        assert ((lab >= 1) & (lab <= 1000)).all()
        seen.append(lab.clone())
    ld.close()
    assert len(set(torch.cat(seen).tolist())) > 4


def test_inference_loader_falls_back_to_train_shards(fake_dir, tmp_path):
    """--forward_only reads the validation shards; a train-only directory still serves it."""
    import make_fake_imagenet

    from azure_hc_intel_tf_amd.data.imagenet import ImageNetLoader

    ld = ImageNetLoader(fake_dir, 4, 32, 3, "cpu", train=False, seed=0, reader_threads=2, decode_threads=2, depth=2)
    assert ld.files and all("validation-" in os.path.basename(f) for f in ld.files)
    ld.close()
    make_fake_imagenet.make(str(tmp_path), shards=2, per_shard=8, subset="train", seed=4)
    ld = ImageNetLoader(str(tmp_path), 4, 32, 3, "cpu", train=False, seed=0, reader_threads=2, decode_threads=2,
                        depth=2)
    assert ld.files and all("train-" in os.path.basename(f) for f in ld.files)
    img = torch.zeros(4, 32, 32, 3)
    lab = torch.zeros(4, dtype=torch.int64)
    ld.next_into(img, lab)
    ld.close()
    assert img.abs().max() <= 1.0 + 1e-6 and img.std() > 0.01


def test_cli_real_data_cpu_end_to_end(fake_dir, tmp_path):
    out = tmp_path / "summary.json"
    cmd = [sys.executable, os.path.join(ROOT, "tf_cnn_benchmarks.py"), "--device=cpu", "--model=trivial",
           "--batch_size=4", "--num_batches=3", "--num_warmup_batches=1", "--display_every=1",
           f"--data_dir={fake_dir}", "--data_name=imagenet", "--image_size=32", f"--json_summary={out}"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "TFRecords" in r.stdout and "total images/sec" in r.stdout
    import json

    s = json.loads(out.read_text())
    assert s["data"] == "imagenet-tfrecord" and s["num_batches"] == 3


def test_native_data_library_under_asan_ubsan(tmp_path):
    """Host sanitizers over the C++ data core (GPU sanitizers are unavailable on the pool):
    ASan + UBSan build driven through corrupted records, junk Example bytes, crop sampling
    and prefetcher start/stop."""
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize_data.sh"), str(tmp_path)], cwd=ROOT,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "sanitize_data: ok" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
