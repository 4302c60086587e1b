"""The reference's two CIFAR-10 CNNs and an MNIST MLP.

Architectures match /root/reference/example/models.py (LeNet :5-23,
AlexNet :25-49) layer for layer, so parameter counts and the flat ravel order
are identical (LeNet 62,006 params; AlexNet 2,472,266).  They are built from
this package's layers, so every GPU op is a native kernel: the convs (implicit
GEMM, or patch matrix + MFMA GEMM for AlexNet's 11x11 stem and both LeNet
convs), the linears (MFMA GEMM), max-pool, dropout, cross-entropy, optimizer;
each ReLU is fused into the epilogue of the conv / linear that produces its
input (``L.fuse_relu``; ReLU commutes with max-pool and with dropout's
non-negative scaling, so LeNet's pool -> ReLU is the same function).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops import functional as DF
from ..ops import layers as L


class LeNet(nn.Module):
    """conv5(3->6) -> pool2 -> relu -> conv5(6->16) -> dropout2d -> pool2 -> relu
    -> fc 400->120 -> relu -> dropout -> fc 120->84 -> relu -> fc 84->10."""

    def __init__(self, num_classes: int = 10):
        super().__init__()
        self.conv1 = L.Conv2d(3, 6, kernel_size=5)
        self.conv2 = L.Conv2d(6, 16, kernel_size=5)
        self.conv2_drop = L.Dropout2d()
        self.fc1_drop = L.Dropout()
        self.fc1 = L.Linear(16 * 5 * 5, 120)
        self.fc2 = L.Linear(120, 84)
        self.fc3 = L.Linear(84, num_classes)

    def forward(self, x):
        # relu(pool(c)) == pool(relu(c)); relu(pool(drop(c))) == pool(drop(relu(c)))
        h = DF.max_pool2d(self.conv1(x, relu=True), 2)
        # the pool writes (c, h, w) order directly: flatten is a view
        h = DF.max_pool2d(self.conv2_drop(self.conv2(h, relu=True)), 2, nchw_out=True)
        h = torch.flatten(h.contiguous(), 1)
        h = self.fc1_drop(self.fc1(h, relu=True))
        h = self.fc2(h, relu=True)
        return self.fc3(h)


class AlexNet(nn.Module):
    """AlexNet adapted to 32x32 inputs: conv11/s4/p5(64) pool, conv5/p2(192) pool,
    conv3(384), conv3(256), conv3(256) pool, linear 256->classes."""

    def __init__(self, num_classes: int = 10):
        super().__init__()
        self.features = nn.Sequential(
            L.Conv2d(3, 64, kernel_size=11, stride=4, padding=5),
            nn.ReLU(inplace=True),
            L.MaxPool2d(kernel_size=2, stride=2),
            L.Conv2d(64, 192, kernel_size=5, padding=2),
            nn.ReLU(inplace=True),
            L.MaxPool2d(kernel_size=2, stride=2),
            L.Conv2d(192, 384, kernel_size=3, padding=1),
            nn.ReLU(inplace=True),
            L.Conv2d(384, 256, kernel_size=3, padding=1),
            nn.ReLU(inplace=True),
            L.Conv2d(256, 256, kernel_size=3, padding=1),
            nn.ReLU(inplace=True),
            L.MaxPool2d(kernel_size=2, stride=2),
        )
        self.classifier = L.Linear(256, num_classes)

    def forward(self, x):
        h = L.fuse_relu(self.features, x)
        return self.classifier(torch.flatten(h.contiguous(), 1))


class MLP(nn.Module):
    """MNIST-shaped MLP (BASELINE.json config #1: 2-worker ASGD over gloo)."""

    def __init__(self, in_features: int = 784, hidden=(512, 256), num_classes: int = 10):
        super().__init__()
        dims = [in_features, *hidden]
        self.layers = nn.ModuleList(L.Linear(a, b) for a, b in zip(dims[:-1], dims[1:]))
        self.head = L.Linear(dims[-1], num_classes)

    def forward(self, x):
        h = torch.flatten(x, 1)
        for lin in self.layers:
            h = lin(h, relu=True)
        return self.head(h)
