#!/usr/bin/env python3
"""Exercise the native data library (TFRecord framing / CRC-32C, tf.Example parse+encode, JPEG
probe, crop windows, multi-threaded prefetcher) WITHOUT torch, so it can run under the
host AddressSanitizer / UndefinedBehaviorSanitizer build (tools/sanitize_data.sh):
corrupted / truncated records, garbage Example bytes and early prefetcher shutdown included."""
import os
import random
import sys
import tempfile

sys.path.insert(0, os.environ.get("HCB_DATA_LIB_DIR", ""))
import _hcb_data as D  # noqa: E402


def main():
    rnd = random.Random(0)
    assert D.crc32c(b"123456789") == 0xE3069283
    tmp = tempfile.mkdtemp()
    files = []
    for s in range(3):
        p = os.path.join(tmp, f"train-{s:05d}-of-00003")
        w = D.RecordWriter(p)
        for i in range(50):
            jpeg = b"\xff\xd8\xff\xc0\x00\x11\x08" + bytes([1, 40, 1, 60, 3]) + bytes(rnd.randrange(256) for _ in range(200))
            w.write(D.encode_example({"image/encoded": [jpeg], "image/class/label": [i + 1],
                                      "image/object/bbox/ymin": [0.1], "image/object/bbox/xmin": [0.2],
                                      "image/object/bbox/ymax": [0.9], "image/object/bbox/xmax": [0.8]}))
        w.close()
        files.append(p)
    # round trip + dims probe
    r = D.RecordReader(files[0], True)
    n = 0
    while True:
        rec = r.next()
        if rec is None:
            break
        ex = D.parse_example(rec)
        assert D.jpeg_dims(ex["image/encoded"][0]) == (296, 316, 3)
        n += 1
    assert n == 50
    # garbage Example bytes must raise, never crash
    for _ in range(2000):
        junk = bytes(rnd.randrange(256) for _ in range(rnd.randrange(1, 64)))
        try:
            D.parse_example(junk)
        except Exception:
            pass
        D.jpeg_dims(junk)
    # corrupted / truncated files raise
    raw = bytearray(open(files[1], "rb").read())
    bad = os.path.join(tmp, "bad.tfrecord")
    open(bad, "wb").write(bytes(raw[: len(raw) // 2 + 5]))  # mid-record
    try:
        rr = D.RecordReader(bad, True)
        while rr.next() is not None:
            pass
        raise SystemExit("truncation not detected")
    except RuntimeError:
        pass
    for seed in range(500):
        y, x, h, w = D.distorted_crop(rnd.randrange(1, 800), rnd.randrange(1, 800), [(0.1, 0.1, 0.9, 0.9)], seed=seed)
        assert h > 0 and w > 0
    # prefetcher: threads, shuffling, epochs, early stop with full queues
    for train in (True, False):
        pf = D.Prefetcher(files, rank=0, world=1, threads=3, shuffle_buffer=16, capacity=32, seed=1, train=train,
                          loop=True)
        for _ in range(20):
            assert len(pf.next(16)) == 16
        pf.stop()
    pf = D.Prefetcher(files, threads=2, shuffle_buffer=8, capacity=8, loop=True)
    pf.next(3)
    del pf  # destructor joins reader threads blocked on a full pool
    print("sanitize_data: ok")


if __name__ == "__main__":
    main()
