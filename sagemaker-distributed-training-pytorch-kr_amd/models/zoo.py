"""Vision model registry used by the DDP image recipes (replaces ``torchvision.models.__dict__``)."""
from __future__ import annotations

import torch.nn as nn

from . import resnet as _resnet
from . import swin as _swin
from .mnist import Net as MnistNet


def available():
    return _resnet.available() + _swin.available() + ["mnist_cnn"]


def create(name: str, num_classes: int = 1000) -> nn.Module:
    if name in _resnet.available():
        return _resnet.resnet(name, num_classes=num_classes)
    if name in _swin.available():
        return _swin.swin(name, num_classes=num_classes)
    if name == "mnist_cnn":
        return MnistNet()
    raise ValueError(f"unknown model '{name}'; available: {available()}")


def reset_classifier(model: nn.Module, num_classes: int):
    """Replace the final classifier so the model predicts ``num_classes`` classes."""
    for attr in ("fc", "head", "classifier"):
        layer = getattr(model, attr, None)
        if isinstance(layer, nn.Linear):
            setattr(model, attr, nn.Linear(layer.in_features, num_classes, bias=layer.bias is not None))
            return model
    raise ValueError("model has no linear classifier named fc/head/classifier")
