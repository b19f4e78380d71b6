"""Model registry: name -> model (tf_cnn_benchmarks ``models/model_config.py`` role,
SURVEY.md §2.2). Names follow ``--model=`` of tf_cnn_benchmarks."""
from __future__ import annotations

from .base import CNNModel
from .resnet import ResNet


def _resnet(depth, version):
    return lambda **kw: ResNet(depth=depth, version=version, **kw)


def _resnet_v2(depth):
    def make(**kw):
        from .resnet import ResNetV2

        return ResNetV2(depth=depth, **kw)

    return make


def _inception3(**kw):
    from .inception import InceptionV3

    return InceptionV3(**kw)


def _trivial(**kw):
    from .trivial import Trivial

    return Trivial(**kw)


def _seq(cls_name, **fixed):
    def make(**kw):
        from . import sequential

        return getattr(sequential, cls_name)(**fixed, **kw)

    return make


_MODELS = {
    "resnet50": _resnet(50, "v1"),
    "resnet50_v1.5": _resnet(50, "v1.5"),
    "resnet101": _resnet(101, "v1"),
    "resnet101_v1.5": _resnet(101, "v1.5"),
    "resnet152": _resnet(152, "v1"),
    "resnet152_v1.5": _resnet(152, "v1.5"),
    "resnet50_v2": _resnet_v2(50),
    "resnet101_v2": _resnet_v2(101),
    "resnet152_v2": _resnet_v2(152),
    "inception3": _inception3,
    "trivial": _trivial,
    "vgg11": _seq("VGG", depth=11),
    "vgg16": _seq("VGG", depth=16),
    "vgg19": _seq("VGG", depth=19),
    "alexnet": _seq("AlexNet"),
    "overfeat": _seq("OverFeat"),
    "lenet": _seq("LeNet"),
    "googlenet": _seq("GoogLeNet"),
}


def model_names():
    return sorted(_MODELS)


def create_model(name: str, **kw) -> CNNModel:
    if name not in _MODELS:
        raise ValueError(f"unknown model {name!r}; available: {', '.join(model_names())}")
    return _MODELS[name](**kw)


__all__ = ["create_model", "model_names", "CNNModel", "ResNet"]
