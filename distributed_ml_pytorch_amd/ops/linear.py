"""Fully-connected layer with arena-direct fp32 weight gradients.

Forward and data gradient are plain bf16 GEMMs (hipBLASLt through
``F.linear`` / ``matmul``) on the arena's bf16 weight shadow, so no per-step
cast.  The weight gradient is ONE bf16 x bf16 -> fp32 GEMM that accumulates
straight into the fp32 arena gradient view -- the native MFMA wgrad kernel
(a 1x1 convolution's weight gradient) when the dims are multiples of 64,
else ``addmm`` with an fp32 ``out_dtype`` and ``beta = 1``: no bf16
weight-gradient tensor, no mixed-dtype add kernel, no AccumulateGrad.  On the
native path the bias gradient is summed by the same kernel from the dY tiles it
already stages; otherwise it is one native column-sum pass (``csrc/linear.hip``)
adding straight into the fp32 arena view.  Both fire the parameter's grad-ready
hook (bucketed all-reduce in sync DP) as soon as they land.

Parity: the reference's ``nn.Linear`` layers (/root/reference/example/models.py
LeNet/AlexNet/MLP heads) in fp32; here bf16 compute with fp32 master weights.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch.autograd import Function

from ._ext import native
from .functional import _notify


_COLSUM_SCRATCH: dict = {}


def colsum_scratch(device, n: int) -> torch.Tensor:
    """Per-device zeroed fp32 slot scratch of the bias-grad column sum
    (csrc/linear.hip); every call leaves it zeroed, and calls on one stream are
    ordered, so all layers share it."""
    need = native().colsum_num_slots() * n
    buf = _COLSUM_SCRATCH.get(device)
    if buf is None or buf.numel() < need:
        buf = torch.zeros(max(need, native().colsum_num_slots() * 4096), dtype=torch.float32,
                          device=device)
        _COLSUM_SCRATCH[device] = buf
    return buf


def bias_grad_acc(dy, out):
    """``out += dy`` summed over every dim but the channel/last one (native, one pass)."""
    n = out.numel()
    native().colsum_acc(dy, out, colsum_scratch(dy.device, n))


def _arena_grad(p):
    if p is None or not p.requires_grad or not getattr(p, "_dmp_arena", False):
        return None
    g = p.grad
    if g is None:
        return None
    if g.dim() == 4 and g.is_contiguous(memory_format=torch.channels_last):
        # conv weight used as a GEMM (patch embedding): [Cout, kh*kw*Cin] view
        return g.permute(0, 2, 3, 1).reshape(g.shape[0], -1)
    return g if g.is_contiguous() else None


def _native_wgrad_ok(dy2, x2) -> bool:
    M, N = dy2.shape
    K = x2.shape[1]
    return (dy2.dtype == torch.bfloat16 and x2.dtype == torch.bfloat16 and N % 64 == 0
            and K % 64 == 0 and M * max(N, K) * 2 < (1 << 30)
            and dy2.is_contiguous() and x2.is_contiguous())


def _native_wgrad(dy2, x2, g, gb=None):
    """g[N, K] += dy2^T @ x2 as a 1x1 convolution weight gradient on the native
    MFMA wgrad kernel (csrc/conv_wgrad.hip): fp32 atomics straight into the
    arena.  Measured against hipBLASLt's fp32-output addmm on the ViT-B/16
    shapes (scripts/linear_vs_conv1x1.py, profiles/linear_vs_conv1x1_r1.txt):
    1.1-2x faster; forward / dgrad stay on hipBLASLt (it wins those).
    ``gb``: optional fp32 [N] bias gradient, accumulated by the same kernel from
    the dY tiles it already stages (no separate column-sum pass over dY)."""
    from .conv import _wgrad_cfg

    M, N = dy2.shape
    K = x2.shape[1]
    dy4 = dy2.view(M, 1, 1, N).permute(0, 3, 1, 2)     # NCHW view of NHWC memory
    x4 = x2.view(M, 1, 1, K).permute(0, 3, 1, 2)
    g4 = g.view(N, K, 1, 1)
    cfg = _wgrad_cfg(dy4, x4, (N, K, 1, 1), 1, 0)
    native().conv_wgrad(dy4, x4, g4, 1, 0, cfg, gb)


class _ArenaLinear(Function):
    @staticmethod
    def forward(ctx, x, w16, b16, w, b):
        ctx.save_for_backward(x, w16)
        ctx.params = (w, b)
        return F.linear(x, w16, b16)

    @staticmethod
    def backward(ctx, dy):
        x, w16 = ctx.saved_tensors
        w, b = ctx.params
        K, N = x.shape[-1], dy.shape[-1]
        dy2 = dy.reshape(-1, N)
        x2 = x.reshape(-1, K)
        dx = (dy2 @ w16).view(x.shape) if ctx.needs_input_grad[0] else None
        gw = gb = None
        g = _arena_grad(w)
        bias_done = False
        if g is not None:
            if _native_wgrad_ok(dy2, x2):
                gbias = _arena_grad(b) if (b is not None and b.requires_grad) else None
                _native_wgrad(dy2, x2, g, gbias)
                bias_done = gbias is not None
            else:
                torch.ops.aten.addmm.dtype_out(g, dy2.t(), x2, torch.float32, out=g)
            _notify(w)
        elif w is not None and w.requires_grad:
            gw = torch.ops.aten.mm.dtype(dy2.t(), x2, torch.float32).to(w.dtype)
            if w.dim() == 4:                     # patch embedding: (kh, kw, Cin) columns
                gw = gw.view(w.shape[0], w.shape[2], w.shape[3], w.shape[1]).permute(0, 3, 1, 2)
        if b is not None and b.requires_grad:
            g = _arena_grad(b)
            vec = dy2.dtype == torch.bfloat16 and N % 8 == 0    # 16-B column chunks
            if g is not None:
                if bias_done:
                    pass                         # summed by the weight-gradient kernel
                elif vec:
                    bias_grad_acc(dy2, g)        # one pass straight into the arena
                else:
                    g.add_(dy2.sum(0, dtype=torch.float32))
                _notify(b)
            else:
                col = torch.zeros(N, dtype=torch.float32, device=dy.device)
                if vec:
                    bias_grad_acc(dy2, col)
                else:
                    col += dy2.sum(0, dtype=torch.float32)
                gb = col.to(b.dtype)
        return dx, None, None, gw, gb


def arena_linear_ok(x, w, b) -> bool:
    """The weight (and bias) live in an arena with a bf16 shadow matching ``x``."""
    if not (x.is_cuda and x.dtype == torch.bfloat16 and torch.is_grad_enabled()):
        return False
    w16 = getattr(w, "_dmp_w16", None)
    if w16 is None or w16.dtype != x.dtype or not w16.is_contiguous():
        return False
    return b is None or getattr(b, "_dmp_w16", None) is not None


def linear(x, w, b):
    w16 = w._dmp_w16
    b16 = b._dmp_w16 if b is not None else None
    return _ArenaLinear.apply(x, w16, b16, w, b)


def patch_embed_ok(x, w, b, patch: int) -> bool:
    """Non-overlapping ``patch`` x ``patch`` conv whose weight lives in an arena
    with a channels-last bf16 shadow: computable as one GEMM on patch rows."""
    if not (x.is_cuda and x.dtype == torch.bfloat16 and torch.is_grad_enabled()
            and x.dim() == 4 and x.shape[2] % patch == 0 and x.shape[3] % patch == 0):
        return False
    w16 = getattr(w, "_dmp_w16", None)
    if w16 is None or w16.dtype != x.dtype or not w16.is_contiguous(
            memory_format=torch.channels_last):
        return False
    return b is None or getattr(b, "_dmp_w16", None) is not None


def patch_embed(x, w, b, patch: int):
    """ViT patch embedding (stride = kernel = ``patch`` conv) as one GEMM:
    ``[B, C, H, W] -> [B, (H/p)(W/p), Cout]`` tokens.  The patch rows are
    gathered in the weight's physical (kh, kw, Cin) order, so the channels-last
    arena shadow is the GEMM's [Cout, K] operand as-is, and the weight gradient
    lands in the arena through the native wgrad kernel like any linear layer.
    No input gradient (pixels), so no dgrad GEMM.  Replaces a library conv
    forward + backward-weights pair."""
    B, C, H, W = x.shape
    gh, gw = H // patch, W // patch
    xp = (x.reshape(B, C, gh, patch, gw, patch).permute(0, 2, 4, 3, 5, 1)
          .reshape(B, gh * gw, patch * patch * C))
    w16 = w._dmp_w16.permute(0, 2, 3, 1).reshape(w.shape[0], -1)
    b16 = b._dmp_w16 if b is not None else None
    return _ArenaLinear.apply(xp, w16, b16, w, b)
