"""gfx950 HIP ops: autograd functions and nn layers."""
from . import functional
from ._ext import available as native_available, native
from .functional import (batch_norm_act, compute_weight, global_avg_pool, max_pool2d,
                         softmax_cross_entropy)
from .layers import (BatchNorm1d, BatchNorm2d, Conv2d, GlobalAvgPool, Linear, MaxPool2d, ReLU)

__all__ = [
    "functional", "native", "native_available", "batch_norm_act", "compute_weight",
    "global_avg_pool", "max_pool2d", "softmax_cross_entropy", "BatchNorm1d", "BatchNorm2d",
    "Conv2d", "GlobalAvgPool", "Linear", "MaxPool2d", "ReLU",
]
