"""Model zoo: MobileNetV2 (CIFAR, with/without BN), ResNet-18..152, ViT-B/16."""
from __future__ import annotations

from typing import Callable, Dict

import torch.nn as nn

from .mobilenetv2 import (HeadPool, InvertedResidual, MobileNetV2, mobilenet_v2, mobilenet_v2_224,
                          mobilenet_v2_nobn)
from .resnet import BasicBlock, Bottleneck, ResNet, resnet18, resnet34, resnet50, resnet101, resnet152
from .vit import VisionTransformer, vit_b_16, vit_tiny

MODELS: Dict[str, Callable[..., nn.Module]] = {
    "mobilenetv2": mobilenet_v2,
    "mobilenetv2_nobn": mobilenet_v2_nobn,
    "mobilenetv2_224": mobilenet_v2_224,
    "resnet18": resnet18,
    "resnet34": resnet34,
    "resnet50": resnet50,
    "resnet101": resnet101,
    "resnet152": resnet152,
    "vit_b_16": vit_b_16,
    "vit_tiny": vit_tiny,
}

# Default input geometry per model (C, H, W) and class count.
INPUT_SHAPES = {
    "mobilenetv2": ((3, 32, 32), 10),
    "mobilenetv2_nobn": ((3, 32, 32), 10),
    "mobilenetv2_224": ((3, 224, 224), 1000),
    "resnet18": ((3, 224, 224), 1000),
    "resnet34": ((3, 224, 224), 1000),
    "resnet50": ((3, 224, 224), 1000),
    "resnet101": ((3, 224, 224), 1000),
    "resnet152": ((3, 224, 224), 1000),
    "vit_b_16": ((3, 224, 224), 1000),
    "vit_tiny": ((3, 32, 32), 10),
}


def build_model(name: str, **kw) -> nn.Module:
    try:
        return MODELS[name](**kw)
    except KeyError:
        raise ValueError(f"unknown model {name!r}; choose from {sorted(MODELS)}") from None


__all__ = ["MODELS", "INPUT_SHAPES", "build_model", "MobileNetV2", "InvertedResidual", "HeadPool",
           "mobilenet_v2", "mobilenet_v2_nobn", "mobilenet_v2_224", "ResNet", "BasicBlock", "Bottleneck", "resnet18",
           "resnet34", "resnet50", "resnet101", "resnet152", "VisionTransformer", "vit_b_16",
           "vit_tiny"]
