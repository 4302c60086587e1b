"""2-D convolution dispatch.

Native path: NHWC bf16 implicit-GEMM on MFMA (``csrc/conv.hip``) for the
shapes it supports; everything else goes to ``F.conv2d`` in channels_last.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

_NATIVE_CONV = None  # resolved lazily; set by ops.conv_native when built


def conv2d(x, w, b, stride, padding, dilation, groups, master=None):
    if x.is_cuda and x.dim() == 4:
        x = x.contiguous(memory_format=torch.channels_last)
        if _NATIVE_CONV is not None:
            y = _NATIVE_CONV(x, w, b, stride, padding, dilation, groups, master)
            if y is not None:
                return y
    return F.conv2d(x, w, b, stride, padding, dilation, groups)
