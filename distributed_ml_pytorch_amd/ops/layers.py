"""nn.Module layers that route to the gfx950 kernels on GPU.

They subclass the stock torch modules so state_dicts, initialisation and
parameter order (the ravel order of the reference's serialization, see
``utils/serialization.py``) are unchanged.  Compute dtype follows the input:
fp32 masters are cast through the arena's bf16 shadow (``compute_weight``).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import functional as DF
from ._policy import stock_gpu
from .conv import (bn_slot_buffer, conv2d as _conv2d, im2col_conv_supported,
                   native_conv_supported, small_conv_supported)
from .linear import arena_linear_ok, linear as _arena_linear


class Conv2d(nn.Conv2d):
    """Conv2d on the native kernels for bf16 GPU input (implicit GEMM / halo
    tiles, the VALU stem kernel, or patch matrix + MFMA GEMM: ``ops.conv``).

    ``emit_bn_stats`` (set by models where a BatchNorm follows) makes the
    native forward also produce the BN partial sums in its epilogue.
    ``relu=True`` fuses a following ReLU into the epilogue.
    """

    emit_bn_stats = False

    def forward(self, x, alias=False, relu: bool = False, stride=None):
        """``alias=True`` returns ``(y, x_alias)``: route the block's shortcut
        through ``x_alias`` and its gradient is added in this conv's dgrad
        (``alias="sub"``: see ``ops.conv.conv2d``).  ``stride`` overrides the
        module's stride (a stride-2 shortcut applied to an already subsampled x)."""
        st = self.stride if stride is None else (stride, stride)
        if x.is_cuda and x.dtype == torch.bfloat16 and (
                native_conv_supported(x, self.weight, st, self.padding, self.dilation,
                                      self.groups)
                or small_conv_supported(x, self.weight, st, self.padding,
                                        self.dilation, self.groups)
                or im2col_conv_supported(x, self.weight, st, self.padding,
                                         self.dilation, self.groups)):
            want = self.emit_bn_stats and self.training and not relu
            slots = bn_slot_buffer(self, "_dmp_slots", self.out_channels, x.device) if want else None
            return _conv2d(x, None, self.bias, st, self.padding, self.dilation,
                           self.groups, master=self.weight, want_stats=want, slots=slots,
                           alias=alias, relu=relu)
        w = DF.compute_weight(self.weight, x.dtype)
        b = DF.compute_weight(self.bias, x.dtype)
        return _conv2d(x, w, b, st, self.padding, self.dilation, self.groups,
                       alias=alias, relu=relu)


class Linear(nn.Linear):
    def forward(self, x, relu: bool = False):
        if arena_linear_ok(x, self.weight, self.bias):
            return _arena_linear(x, self.weight, self.bias, relu)
        stock_gpu("linear", x, reason=f"input {tuple(x.shape)} {x.dtype}, weight "
                  f"{tuple(self.weight.shape)} (no bf16 arena shadow)")
        w = DF.compute_weight(self.weight, x.dtype)
        b = DF.compute_weight(self.bias, x.dtype)
        y = F.linear(x, w, b)
        return DF.relu(y) if relu else y


def _bn_slots(mod, x):
    if not x.is_cuda:
        return None
    return (bn_slot_buffer(mod, "_dmp_fslots", mod.num_features, x.device),
            bn_slot_buffer(mod, "_dmp_bslots", mod.num_features, x.device, fresh=False))


class BatchNorm2d(nn.BatchNorm2d):
    """BatchNorm with optional fused residual-add and ReLU epilogue."""

    _slots = _bn_slots

    def __init__(self, num_features, eps=1e-5, momentum=0.1, relu: bool = False, **kw):
        super().__init__(num_features, eps=eps, momentum=momentum, **kw)
        self.relu = relu

    def forward(self, x, residual=None):
        use_batch = self.training or not self.track_running_stats
        return DF.batch_norm_act(
            x, self.weight, self.bias,
            self.running_mean if self.track_running_stats else None,
            self.running_var if self.track_running_stats else None,
            use_batch, 0.1 if self.momentum is None else self.momentum, self.eps,
            relu=self.relu, residual=residual, slots=self._slots(x))


class BatchNorm1d(nn.BatchNorm1d):
    _slots = _bn_slots

    def __init__(self, num_features, eps=1e-5, momentum=0.1, relu: bool = False, **kw):
        super().__init__(num_features, eps=eps, momentum=momentum, **kw)
        self.relu = relu

    def forward(self, x, residual=None):
        use_batch = self.training or not self.track_running_stats
        return DF.batch_norm_act(
            x, self.weight, self.bias,
            self.running_mean if self.track_running_stats else None,
            self.running_var if self.track_running_stats else None,
            use_batch, 0.1 if self.momentum is None else self.momentum, self.eps,
            relu=self.relu, residual=residual, slots=self._slots(x))


class MaxPool2d(nn.MaxPool2d):
    def native_params(self):
        """(k, s, p) as ints when the native floor-mode square pool applies, else
        None (ceil_mode, dilation, or a non-square kernel / stride / padding)."""
        def one(v):
            if isinstance(v, int):
                return v
            v = tuple(v)
            return v[0] if len(v) == 2 and v[0] == v[1] else None
        k, s, p = one(self.kernel_size), one(self.stride), one(self.padding)
        d = one(self.dilation)
        if self.ceil_mode or d != 1 or None in (k, s, p):
            return None
        return k, s, p

    def forward(self, x):
        kp = self.native_params()
        if kp is None:
            stock_gpu("max_pool2d", x, reason="ceil_mode / dilation / non-square window")
            return super().forward(x)
        return DF.max_pool2d(x, *kp)


class GlobalAvgPool(nn.Module):
    def forward(self, x):
        return DF.global_avg_pool(x)


class ReLU(nn.ReLU):
    """ReLU on the native mask kernel for bf16 GPU tensors (models fuse it into
    the producing conv / linear epilogue where they can: ``fuse_relu``)."""

    def forward(self, x):
        return DF.relu(x)


def fuse_relu(seq, x):
    """Run an nn.Sequential, folding every ReLU that directly follows a Conv2d /
    Linear of this package into that layer's epilogue (the ReLU modules stay in
    the Sequential, so parameter names and state_dict keys are unchanged)."""
    mods = list(seq)
    i = 0
    while i < len(mods):
        m = mods[i]
        nxt = mods[i + 1] if i + 1 < len(mods) else None
        if isinstance(m, (Conv2d, Linear)) and isinstance(nxt, nn.ReLU):
            x = m(x, relu=True)
            i += 2
            continue
        x = m(x)
        i += 1
    return x


class _DropoutBase(nn.Module):
    channelwise = False

    def __init__(self, p: float = 0.5, seed: int | None = None):
        super().__init__()
        if not 0.0 <= p < 1.0:
            raise ValueError(f"dropout probability must be in [0, 1), got {p}")
        self.p = p
        self.seed = int(torch.randint(0, 2**62, (1,)).item()) if seed is None else int(seed)
        self._state = None

    def forward(self, x):
        state = None
        if x.is_cuda:
            if self._state is None or self._state.device != x.device:
                # [Philox offset, arrival ticket of the launch advancing it]
                self._state = torch.zeros(2, dtype=torch.int64, device=x.device)
            state = self._state
        return DF.dropout(x, self.p, self.training, self.channelwise, state, self.seed)

    def extra_repr(self):
        return f"p={self.p}"


class Dropout(_DropoutBase):
    """Element-wise dropout on the Philox kernel (``csrc/dropout.hip``)."""


class Dropout2d(_DropoutBase):
    """Channel (plane) dropout on the Philox kernel."""

    channelwise = True

