"""ResNet family for BASELINE.json configs #2-#4 (ResNet-18 ASGD, ResNet-50 sync DP).

Not present in the reference (its models are LeNet/AlexNet only);
the north-star metric is ResNet-18 samples/s.  Two stems:

* ``cifar``    : conv3x3(64) stride 1, no max-pool (32x32 inputs). ResNet-18 ->
  11,173,962 parameters, the count SURVEY §5.8 prices the messages with.
* ``imagenet`` : conv7x7/s2 + maxpool3/s2 (224x224 inputs). ResNet-50 ->
  25,557,032 parameters.

Every conv is followed by a fused BN(+residual)(+ReLU) kernel pair; the
block output ``relu(bn2(conv2(h)) + shortcut)`` is ONE kernel on GPU.  In eval
mode under ``no_grad`` (the reference's evaluation loop) every BatchNorm is
folded into its conv instead (ops/eval_fold.py): one launch per conv, none
per BatchNorm.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from ..ops import layers as L
from ..ops.eval_fold import conv_bn, fold_enabled
from ..ops.functional import bn_relu_maxpool, bn_relu_maxpool_ok, mark_residual_only
from ..ops.linear import gap_linear, gap_linear_ok


# 1x1 / stride-2 shortcuts on conv1's subsampled alias (DMP_SC_SUB=0: full-res
# alias and a stride-2 shortcut conv, for A/B)
_SC_SUB = os.environ.get("DMP_SC_SUB", "1") != "0"


def _sc_sub(shortcut) -> bool:
    """A 1x1 / stride-2 / unpadded shortcut conv that can run on x[:, :, ::2, ::2]."""
    return (shortcut is not None and _SC_SUB and shortcut[0].kernel_size == (1, 1)
            and shortcut[0].stride == (2, 2) and shortcut[0].padding == (0, 0))


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin: int, planes: int, stride: int = 1):
        super().__init__()
        self.conv1 = L.Conv2d(cin, planes, 3, stride=stride, padding=1, bias=False)
        self.bn1 = L.BatchNorm2d(planes, relu=True)
        self.conv2 = L.Conv2d(planes, planes, 3, stride=1, padding=1, bias=False)
        self.bn2 = L.BatchNorm2d(planes, relu=True)
        self.shortcut = None
        if stride != 1 or cin != planes:
            self.shortcut = nn.Sequential(
                L.Conv2d(cin, planes, 1, stride=stride, bias=False), L.BatchNorm2d(planes))

    def _forward_folded(self, x):
        h = conv_bn(x, self.conv1, self.bn1)
        if h is None:
            return None
        sc = x if self.shortcut is None else conv_bn(x, self.shortcut[0], self.shortcut[1])
        if sc is None:
            return None
        return conv_bn(h, self.conv2, self.bn2, residual=sc)

    def forward(self, x):
        if fold_enabled(x, self):
            y = self._forward_folded(x)
            if y is not None:
                return y
        # the shortcut reads x through conv1's alias: its gradient is summed into
        # x's gradient by conv1's dgrad epilogue (no autograd add).  A 1x1 /
        # stride-2 shortcut takes conv1's subsampled alias x[:, :, ::2, ::2] and
        # runs at stride 1 (a plain GEMM; its gradient lands on conv1's stride-2
        # dgrad parity class (0, 0)) when conv1 is native; else the full x.
        sub = self.conv1.stride == (2, 2) and _sc_sub(self.shortcut)
        h, xa = self.conv1(x, alias="sub" if sub else True)
        h = self.bn1(h)
        if self.shortcut is None:
            sc = xa
        elif sub and xa.shape[-1] != x.shape[-1]:
            sc = self.shortcut[1](self.shortcut[0](xa, stride=1))
        else:
            sc = self.shortcut(xa)
        # sc feeds only bn2: its backward may hand dY over unmasked (deferred
        # residual mask) to conv1's dgrad epilogue or the shortcut BN.  Not when sc
        # IS x (conv1 off the native path hands x itself back): x also feeds
        # conv1, autograd would sum the tagged hand-off with conv1's dx and drop
        # the owed mask
        return self.bn2(self.conv2(h), residual=sc if sc is x else mark_residual_only(sc))


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin: int, planes: int, stride: int = 1):
        super().__init__()
        out = planes * self.expansion
        self.conv1 = L.Conv2d(cin, planes, 1, bias=False)
        self.bn1 = L.BatchNorm2d(planes, relu=True)
        self.conv2 = L.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = L.BatchNorm2d(planes, relu=True)
        self.conv3 = L.Conv2d(planes, out, 1, bias=False)
        self.bn3 = L.BatchNorm2d(out, relu=True)
        self.shortcut = None
        if stride != 1 or cin != out:
            self.shortcut = nn.Sequential(
                L.Conv2d(cin, out, 1, stride=stride, bias=False), L.BatchNorm2d(out))

    def _forward_folded(self, x):
        h = conv_bn(x, self.conv1, self.bn1)
        h = conv_bn(h, self.conv2, self.bn2) if h is not None else None
        if h is None:
            return None
        sc = x if self.shortcut is None else conv_bn(x, self.shortcut[0], self.shortcut[1])
        if sc is None:
            return None
        return conv_bn(h, self.conv3, self.bn3, residual=sc)

    def forward(self, x):
        if fold_enabled(x, self):
            y = self._forward_folded(x)
            if y is not None:
                return y
        # a 1x1 / stride-2 shortcut reads conv1's subsampled alias and runs at
        # stride 1 (a GEMM); its gradient is added onto dX's even pixels after
        # conv1's dgrad (see BasicBlock)
        sub = _sc_sub(self.shortcut)
        h, xa = self.conv1(x, alias="sub" if sub else True)
        h = self.bn2(self.conv2(self.bn1(h)))
        if self.shortcut is None:
            sc = xa
        elif sub and xa.shape[-1] != x.shape[-1]:
            sc = self.shortcut[1](self.shortcut[0](xa, stride=1))
        else:
            sc = self.shortcut(xa)
        # sc feeds only bn3 (deferred residual mask: the identity alias's consumer
        # is conv1's 1x1 GEMM-route dgrad, whose store epilogue applies the mask)
        return self.bn3(self.conv3(h), residual=sc if sc is x else mark_residual_only(sc))


class ResNet(nn.Module):
    def __init__(self, block, layers, num_classes: int = 10, stem: str = "cifar",
                 zero_init_residual: bool = False):
        super().__init__()
        self.stem_kind = stem
        if stem == "cifar":
            self.conv1 = L.Conv2d(3, 64, 3, stride=1, padding=1, bias=False)
            self.pool = None
        elif stem == "imagenet":
            self.conv1 = L.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
            self.pool = L.MaxPool2d(3, stride=2, padding=1)
        else:
            raise ValueError(f"unknown stem {stem!r}")
        self.bn1 = L.BatchNorm2d(64, relu=True)
        cin = 64
        stages = []
        for i, (planes, n) in enumerate(zip((64, 128, 256, 512), layers)):
            blocks = []
            for j in range(n):
                stride = 2 if (i > 0 and j == 0) else 1
                blocks.append(block(cin, planes, stride))
                cin = planes * block.expansion
            stages.append(nn.Sequential(*blocks))
        self.layer1, self.layer2, self.layer3, self.layer4 = stages
        self.avgpool = L.GlobalAvgPool()
        self.linear = L.Linear(cin, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            if isinstance(m, L.Conv2d):
                m.emit_bn_stats = True      # every conv here feeds a BatchNorm
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)
                elif isinstance(m, BasicBlock):
                    nn.init.zeros_(m.bn2.weight)

    def forward(self, x):
        h = conv_bn(x, self.conv1, self.bn1) if fold_enabled(x, self) else None
        pooled = False
        if h is None:
            h = self.conv1(x)
            # ints, floor mode, no dilation: else the separate pool below
            pk = self.pool.native_params() if self.pool is not None else None
            if pk is not None and bn_relu_maxpool_ok(h, self.bn1, *pk):
                h, pooled = bn_relu_maxpool(h, self.bn1, *pk), True   # BN + ReLU + pool fused
            else:
                h = self.bn1(h)
        if self.pool is not None and not pooled:
            h = self.pool(h)
        h = self.layer4(self.layer3(self.layer2(self.layer1(h))))
        if gap_linear_ok(h, self.linear):
            return gap_linear(h, self.linear)     # pool + classifier: one launch each way
        return self.linear(self.avgpool(h))


def resnet18(num_classes: int = 10, stem: str = "cifar", **kw) -> ResNet:
    return ResNet(BasicBlock, (2, 2, 2, 2), num_classes, stem, **kw)


def resnet34(num_classes: int = 10, stem: str = "cifar", **kw) -> ResNet:
    return ResNet(BasicBlock, (3, 4, 6, 3), num_classes, stem, **kw)


def resnet50(num_classes: int = 1000, stem: str = "imagenet", **kw) -> ResNet:
    return ResNet(Bottleneck, (3, 4, 6, 3), num_classes, stem, **kw)


def resnet101(num_classes: int = 1000, stem: str = "imagenet", **kw) -> ResNet:
    return ResNet(Bottleneck, (3, 4, 23, 3), num_classes, stem, **kw)
