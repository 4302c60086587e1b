"""Inference-time BatchNorm folding into the producing convolution.

The reference evaluates on its test set every ``log_interval`` iterations and
at every epoch end (/root/reference/example/main.py:83-93, 110-125).  In eval
mode a BatchNorm is a per-channel affine map of running statistics, so

    relu?(BN(conv(x, W)) [+ residual])  ==  relu?(conv(x, W * s) + t [+ residual])

with ``s = gamma / sqrt(running_var + eps)`` and ``t = beta + (b - mean) * s``:
the conv's own epilogue (fp32 bias, residual addend, ReLU -- csrc/conv.hip)
then IS the BatchNorm.  No statistics, finalize or apply pass runs: one
``bn_fold_weights`` launch per conv rescales the fp32 master weights straight
into a bf16 compute weight (one rounding, as the arena's bf16 shadow), and a
:func:`fold_session` (``Worker.evaluate``) does that once per evaluation pass
instead of per batch.

Used by the ResNet blocks (models/resnet.py) whenever the block is in eval mode
under ``torch.no_grad()`` on a bf16 GPU input; anything else (training, CPU,
fp32 oracle runs, unsupported geometries) takes the regular BatchNorm path.
``DMP_EVAL_FOLD=0`` disables it (A/B).
"""
from __future__ import annotations

import contextlib
import os

import torch

from ._ext import native

_FOLD = os.environ.get("DMP_EVAL_FOLD", "1") != "0"
_SESSION = {"depth": 0, "cache": {}}


@contextlib.contextmanager
def fold_session():
    """Fold every (conv, BN) pair once for a whole evaluation pass: weights and
    running statistics cannot change while it runs under ``no_grad``."""
    _SESSION["depth"] += 1
    try:
        yield
    finally:
        _SESSION["depth"] -= 1
        if _SESSION["depth"] == 0:
            _SESSION["cache"].clear()


def fold_enabled(x, module) -> bool:
    return (_FOLD and not module.training and not torch.is_grad_enabled() and x.is_cuda
            and x.dtype == torch.bfloat16 and x.dim() == 4)


def _foldable(bn) -> bool:
    # running statistics only: a BatchNorm left in train mode inside an eval-mode
    # block normalises with batch statistics, which a fold cannot reproduce
    return (not bn.training and bn.track_running_stats and bn.running_mean is not None
            and bn.running_var is not None)


def _folded(conv, bn):
    key = (id(conv), id(bn))
    hit = _SESSION["cache"].get(key) if _SESSION["depth"] else None
    if hit is not None:
        return hit
    w = conv.weight.detach()
    if w.dtype != torch.float32:
        w = w.float()
    if not (w.is_contiguous(memory_format=torch.channels_last) or w.is_contiguous()):
        w = w.contiguous(memory_format=torch.channels_last)
    g = bn.weight.detach() if bn.weight is not None else None
    b = bn.bias.detach() if bn.bias is not None else None
    cb = conv.bias.detach().float().contiguous() if conv.bias is not None else None
    w16, t32, t16 = native().bn_fold_weights(w, g, b, bn.running_mean, bn.running_var, cb,
                                             float(bn.eps))
    out = {"w16": w16.contiguous(memory_format=torch.channels_last), "t32": t32, "t16": t16}
    if _SESSION["depth"]:
        _SESSION["cache"][key] = out
    return out


def _rows(t):
    t = t.contiguous(memory_format=torch.channels_last)
    return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1])


def conv_bn(x, conv, bn, residual=None):
    """``relu?(bn(conv(x)) [+ residual])`` of an eval-mode pair in ONE native
    conv / GEMM launch (``bn.relu`` says whether a ReLU follows); ``None`` when
    the pair or geometry is not covered (the caller runs the regular path)."""
    from .conv import (_GEMM_ROUTE, _ceil8, _fwd_cfg, _pair, im2col_conv_supported,
                       native_conv_supported, stem_conv_supported)
    from .linear import gemm

    if not _foldable(bn) or conv.groups != 1 or _pair(conv.dilation) != (1, 1):
        return None
    x = x.contiguous(memory_format=torch.channels_last)
    relu = bool(getattr(bn, "relu", False))
    st, pd = _pair(conv.stride)[0], _pair(conv.padding)[0]
    if residual is not None:
        residual = residual.contiguous(memory_format=torch.channels_last)
    f = _folded(conv, bn)
    w16 = f["w16"]
    B, CI, H, W = x.shape
    CO, _, R, S = w16.shape
    if native_conv_supported(x, conv.weight, conv.stride, conv.padding, conv.dilation, 1):
        cfg = _fwd_cfg(x, w16, st, pd)
        if cfg == _GEMM_ROUTE:
            # 1x1 / stride 1 on the GEMM store epilogue: bf16 shift, residual as aux
            y2 = torch.empty(B * H * W, CO, dtype=x.dtype, device=x.device)
            gemm(0, 0, _rows(x), w16.reshape(CO, CI), y2, bias=f["t16"],
                 aux=_rows(residual) if residual is not None else None, relu=relu)
            return y2.view(B, H, W, CO).permute(0, 3, 1, 2)
        y, _, _ = native().conv_fwd(x, w16, st, pd, False, cfg, None, f["t32"], relu, residual)
        return y
    if residual is None and stem_conv_supported(x, conv.weight, conv.stride, conv.padding,
                                                 conv.dilation, 1):
        # ImageNet 7x7/2 stem: the space-to-depth MFMA kernel, shift + ReLU in its epilogue
        return native().stem_fwd(x, w16, False, None, f["t32"], relu)[0]
    if residual is None and im2col_conv_supported(x, conv.weight, conv.stride, conv.padding,
                                                   conv.dilation, 1):
        # stems (3 input channels): patch matrix + GEMM, shift + ReLU in its epilogue
        K = R * S * CI
        Kp = _ceil8(K)
        wp = f.get("wp")
        if wp is None:
            wmat = w16.permute(0, 2, 3, 1).reshape(CO, K)
            wp = wmat if Kp == K else torch.zeros(CO, Kp, dtype=w16.dtype, device=w16.device)
            if Kp != K:
                wp[:, :K] = wmat
            f["wp"] = wp
        cols = native().im2col(x, R, S, st, pd, Kp)
        OH = (H + 2 * pd - R) // st + 1
        OW = (W + 2 * pd - S) // st + 1
        y2 = torch.empty(B * OH * OW, CO, dtype=x.dtype, device=x.device)
        gemm(0, 0, cols, wp, y2, bias=f["t16"], relu=relu)
        return y2.view(B, OH, OW, CO).permute(0, 3, 1, 2)
    return None
