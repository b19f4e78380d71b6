"""Input pipelines: synthetic ImageNet (``trainer.synthetic_batch``, the reference's default
when no ``--data_dir`` is given) and real ImageNet TFRecords (``imagenet.ImageNetLoader``)."""
from .tfrecord import (encode_example, find_shards, imagenet_example, native, parse_example, read_records,
                       write_records)

__all__ = ["encode_example", "find_shards", "imagenet_example", "native", "parse_example", "read_records",
           "write_records", "ImageNetLoader"]


def __getattr__(name):
    if name == "ImageNetLoader":
        from .imagenet import ImageNetLoader

        return ImageNetLoader
    raise AttributeError(name)
