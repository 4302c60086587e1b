"""2-D convolution dispatch.

Native path (``csrc/conv.hip``): NHWC bf16 implicit GEMM on MFMA for
``groups == 1, dilation == 1, CI % 64 == 0, CO % 64 == 0`` (every ResNet conv
except the 3-channel stem, AlexNet conv2-5).  The weight operand is the
arena's bf16 shadow (no per-step cast) and the weight gradient is accumulated
in fp32 straight into the arena grad view (no AccumulateGrad, no cast
kernels).  When the conv feeds a BatchNorm (``emit_bn_stats``) its epilogue
also emits per-block channel sums, so the BN forward skips its statistics
pass over the activation.  Tile configurations are chosen per shape by
timing them on first use (:mod:`.tuner`).

Few-input-channel convolutions (CIFAR-style stems: ``R*S*CI <= 32``,
``CO % 64 == 0``, input not requiring grad) run on the VALU kernels of
``csrc/conv_small.hip`` with the same fused BN-statistics epilogue and direct
fp32 arena weight-gradient accumulation.

Everything else goes to ``F.conv2d`` (MIOpen) in channels_last.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch.autograd import Function

from ._ext import native
from .tuner import TUNER

_NATIVE_ENABLED = True
_CONFIGS = None
_SMALL_MAX_K = 32


def set_native_conv(enabled: bool):
    global _NATIVE_ENABLED
    _NATIVE_ENABLED = bool(enabled)


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


def _configs():
    global _CONFIGS
    if _CONFIGS is None:
        _CONFIGS = [tuple(c) for c in native().conv_configs()]   # (id, BM, BN, BK, threads, NS)
    return _CONFIGS


def _igemm_candidates(out_channels: int):
    return [c[0] for c in _configs() if c[2] <= max(64, out_channels)]


def _wgrad_candidates(K: int):
    """cfg = BNW sel | BP32 << 2 | NS3 << 3 | (min P rows / 512) << 4 (csrc/conv_wgrad.hip)."""
    cands = []
    for sel, bnw in ((1, 64), (2, 128), (3, 192)):
        if K % bnw:
            continue
        for bp32 in (0, 1):
            for ns3 in (0, 1):
                for chunk in (2, 4, 8):          # x512 rows of P per block
                    cands.append(sel | (bp32 << 2) | (ns3 << 3) | (chunk << 4))
    return cands


def _fwd_cfg(x, w16, stride, pad):
    key = ("fwd", *x.shape, w16.shape[0], w16.shape[2], w16.shape[3], stride, pad)
    return TUNER.best(key, lambda c: native().conv_fwd(x, w16, stride, pad, True, c),
                      _igemm_candidates(w16.shape[0]))


def _dgrad_cfg(dy, w16, H, W, stride, pad):
    key = ("dgrad", *dy.shape, w16.shape[1], H, W, w16.shape[2], w16.shape[3], stride, pad)
    return TUNER.best(key, lambda c: native().conv_dgrad(dy, w16, H, W, stride, pad, c),
                      _igemm_candidates(w16.shape[1]))


def _wgrad_cfg(dy, x, shape, stride, pad):
    key = ("wgrad", *x.shape, *shape, stride, pad)
    if key in TUNER.cache or not TUNER.enabled:
        return TUNER.cache.get(key, -1)
    scratch = torch.empty(shape, dtype=torch.float32, device=x.device,
                          memory_format=torch.channels_last).zero_()
    K = shape[1] * shape[2] * shape[3]
    return TUNER.best(key, lambda c: native().conv_wgrad(dy, x, scratch, stride, pad, c),
                      _wgrad_candidates(K))


class _NativeConv(Function):
    @staticmethod
    def forward(ctx, x, w16, master, stride, pad, want_stats):
        # the BN-partials output never receives a gradient: do not let autograd
        # materialise (zero-fill) one for it every backward
        ctx.set_materialize_grads(False)
        cfg = _fwd_cfg(x, w16, stride, pad)
        y, part, _ = native().conv_fwd(x, w16, stride, pad, want_stats, cfg)
        ctx.save_for_backward(x, w16)
        ctx.master = master
        ctx.geom = (x.shape[2], x.shape[3], stride, pad)
        if want_stats:
            ctx.mark_non_differentiable(part)
            return y, part
        return y, None

    @staticmethod
    def backward(ctx, dy, _dpart):
        if dy is None:
            return None, None, None, None, None, None
        x, w16 = ctx.saved_tensors
        H, W, stride, pad = ctx.geom
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = None
        master = ctx.master
        if ctx.needs_input_grad[0]:
            cfg = _dgrad_cfg(dy, w16, H, W, stride, pad)
            wt = None
            ref = getattr(master, "_dmp_arena_ref", None)
            arena = ref() if ref is not None else None
            shadow = getattr(master, "_dmp_w16", None)
            if arena is not None and shadow is not None and shadow.data_ptr() == w16.data_ptr():
                wt = arena.transposed_conv_shadow(master)
            dx = native().conv_dgrad(dy, w16, H, W, stride, pad, cfg, wt)
        gw = None
        if master is not None and master.requires_grad:
            wcfg = _wgrad_cfg(dy, x, tuple(master.shape), stride, pad)
            g = master.grad if getattr(master, "_dmp_arena", False) else None
            if g is not None and g.is_contiguous(memory_format=torch.channels_last):
                native().conv_wgrad(dy, x, g, stride, pad, wcfg)
                cb = getattr(master, "_dmp_grad_ready", None)
                if cb is not None:
                    cb(master)
            else:
                gw = torch.zeros(tuple(master.shape), dtype=torch.float32, device=x.device)
                gw = gw.contiguous(memory_format=torch.channels_last)
                native().conv_wgrad(dy, x, gw, stride, pad, wcfg)
                gw = gw.to(master.dtype)
        return dx, None, gw, None, None, None


class _SmallConv(Function):
    """Stem conv: forward + weight gradient only (the input is data)."""

    @staticmethod
    def forward(ctx, x, w16, master, stride, pad, want_stats):
        ctx.set_materialize_grads(False)
        y, part, _ = native().conv_small_fwd(x, w16, stride, pad, want_stats)
        ctx.save_for_backward(x)
        ctx.master = master
        ctx.geom = (stride, pad)
        if want_stats:
            ctx.mark_non_differentiable(part)
            return y, part
        return y, None

    @staticmethod
    def backward(ctx, dy, _dpart):
        if dy is None:
            return None, None, None, None, None, None
        (x,) = ctx.saved_tensors
        stride, pad = ctx.geom
        master = ctx.master
        gw = None
        if master is not None and master.requires_grad:
            g = master.grad if getattr(master, "_dmp_arena", False) else None
            if g is not None and g.is_contiguous(memory_format=torch.channels_last):
                native().conv_small_wgrad(dy, x, g, stride, pad)
                cb = getattr(master, "_dmp_grad_ready", None)
                if cb is not None:
                    cb(master)
            else:
                gw = torch.empty(tuple(master.shape), dtype=torch.float32, device=x.device,
                                 memory_format=torch.channels_last).zero_()
                native().conv_small_wgrad(dy, x, gw, stride, pad)
                gw = gw.to(master.dtype)
        return None, None, gw, None, None, None


def small_conv_supported(x, weight, stride, padding, dilation, groups) -> bool:
    if not (_NATIVE_ENABLED and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4):
        return False
    if x.requires_grad or groups != 1 or _pair(dilation) != (1, 1):
        return False
    st, pd = _pair(stride), _pair(padding)
    if st[0] != st[1] or pd[0] != pd[1] or not isinstance(pd[0], int):
        return False
    co, ci, r, s = weight.shape
    # VALU kernels: a win over MIOpen only while K = R*S*CI is tiny (CIFAR-style
    # 3x3x3 stems); 7x7 / 11x11 stems stay on MIOpen's MFMA path
    return co % 64 == 0 and r * s * ci <= _SMALL_MAX_K


def native_conv_supported(x, weight, stride, padding, dilation, groups) -> bool:
    if not (_NATIVE_ENABLED and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4):
        return False
    if groups != 1 or _pair(dilation) != (1, 1):
        return False
    st, pd = _pair(stride), _pair(padding)
    if st[0] != st[1] or pd[0] != pd[1] or not isinstance(pd[0], int):
        return False
    co, ci = weight.shape[0], weight.shape[1]
    return ci % 64 == 0 and co % 64 == 0


def conv2d(x, w, b, stride, padding, dilation, groups, master=None, want_stats=False):
    """Returns ``y`` (with BN partials attached as ``y._dmp_bn_part`` when ``want_stats``)."""
    if x.is_cuda and x.dim() == 4:
        x = x.contiguous(memory_format=torch.channels_last)
        if master is not None and b is None and native_conv_supported(
                x, master, stride, padding, dilation, groups):
            w16 = getattr(master, "_dmp_w16", None)
            if w16 is None or not w16.is_contiguous(memory_format=torch.channels_last):
                w16 = master.detach().to(torch.bfloat16).contiguous(
                    memory_format=torch.channels_last)
            y, part = _NativeConv.apply(x, w16, master, _pair(stride)[0], _pair(padding)[0],
                                        bool(want_stats))
            if part is not None:
                y._dmp_bn_part = part
            return y
        if master is not None and b is None and small_conv_supported(
                x, master, stride, padding, dilation, groups):
            w16 = getattr(master, "_dmp_w16", None)
            if w16 is None or not w16.is_contiguous(memory_format=torch.channels_last):
                w16 = master.detach().to(torch.bfloat16).contiguous(
                    memory_format=torch.channels_last)
            y, part = _SmallConv.apply(x, w16, master, _pair(stride)[0], _pair(padding)[0],
                                       bool(want_stats))
            if part is not None:
                y._dmp_bn_part = part
            return y
    return F.conv2d(x, w, b, stride, padding, dilation, groups)
