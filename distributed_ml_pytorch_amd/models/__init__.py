"""Model zoo: the reference's LeNet/AlexNet plus the BASELINE.json families."""
from __future__ import annotations

from .cnn import MLP, AlexNet, LeNet
from .resnet import ResNet, resnet18, resnet34, resnet50, resnet101
from .vit import VisionTransformer, vit_b16, vit_tiny

# name -> (constructor, input shape (C,H,W), num_classes)
REGISTRY = {
    "mlp": (lambda nc=10: MLP(num_classes=nc), (1, 28, 28), 10),
    "lenet": (lambda nc=10: LeNet(nc), (3, 32, 32), 10),
    "alexnet": (lambda nc=10: AlexNet(nc), (3, 32, 32), 10),
    "resnet18": (lambda nc=10: resnet18(nc, stem="cifar"), (3, 32, 32), 10),
    "resnet34": (lambda nc=10: resnet34(nc, stem="cifar"), (3, 32, 32), 10),
    "resnet50": (lambda nc=1000: resnet50(nc, stem="imagenet"), (3, 224, 224), 1000),
    "resnet50_cifar": (lambda nc=10: resnet50(nc, stem="cifar"), (3, 32, 32), 10),
    "resnet101": (lambda nc=1000: resnet101(nc, stem="imagenet"), (3, 224, 224), 1000),
    "vit_b16": (lambda nc=1000: vit_b16(nc), (3, 224, 224), 1000),
    "vit_tiny": (lambda nc=10: vit_tiny(nc), (3, 32, 32), 10),
}


def build_model(name: str, num_classes: int | None = None):
    """Return ``(model, input_shape, num_classes)`` for a registry name."""
    key = name.lower().replace("-", "_").replace("/", "")
    if key == "vit_b_16":
        key = "vit_b16"
    if key not in REGISTRY:
        raise KeyError(f"unknown model {name!r}; choose from {sorted(REGISTRY)}")
    ctor, shape, nc = REGISTRY[key]
    nc = nc if num_classes is None else num_classes
    return ctor(nc), shape, nc


__all__ = ["MLP", "AlexNet", "LeNet", "ResNet", "resnet18", "resnet34", "resnet50", "resnet101",
           "VisionTransformer", "vit_b16", "vit_tiny", "REGISTRY", "build_model"]
