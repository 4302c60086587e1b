"""2-D convolution dispatch.

Native path (``csrc/conv.hip``): NHWC bf16 implicit GEMM on MFMA for
``groups == 1, dilation == 1, CI % 64 == 0, CO % 64 == 0`` (every ResNet conv
except the 3-channel stem, AlexNet conv2-5), optional fp32 bias added in the
epilogue (AlexNet; reference convs carry biases, /root/reference/example/models.py:28-38).  The weight operand is the
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

Every other bf16 GPU conv (few input / output channels, large windows:
AlexNet's 11x11/s4 stem, the LeNet convs, the ResNet-50 7x7 stem) runs as a
native patch matrix (``csrc/im2col.hip``) on the native MFMA GEMM
(``csrc/gemm.hip``) with bias / ReLU in its epilogue.  ``F.conv2d`` only for
CPU / fp32 inputs.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F
from torch.autograd import Function

from ._ext import native
from ._policy import stock_gpu
from .functional import (DEFER_RES_STATS, apply_bitmask, deferred_mask, is_relu_masked,
                         resolve_deferred, set_nonneg)
from .tuner import TUNER

_NATIVE_ENABLED = True
_CONFIGS = None
_SMALL_MAX_K = 32
# few-input-channel stems: "small" = the VALU kernels of conv_small.hip (BN
# statistics in the epilogue), "im2col" = patch matrix + MFMA GEMM
_STEM = os.environ.get("DMP_STEM", "small")

# Weight gradients on a side HIP stream.  A layer's wgrad depends only on its
# dY and X, and nothing in the rest of the backward depends on it (it lands in
# the fp32 grad arena), so it runs concurrently with the dgrad -> BN-backward
# chain of the layers below: the MFMA-bound wgrad fills the CUs that the
# latency-bound BN reductions / finalizes and the small-grid layer-4 convs
# leave idle.  The side stream is joined back (current stream waits on it) by
# an autograd end-of-backward callback, so callers -- including hipGraph
# capture -- see an ordinary single-stream backward.  Disabled for parameters
# with a grad-ready hook (sync-DP bucket all-reduce orders on the current
# stream).  Opt-in (DMP_WGRAD_STREAM=1): measured on ResNet-18/CIFAR bs256 the
# concurrent wgrad grids delay the single-block BN finalize kernels on the
# critical path (bwd finalize 96 -> 244 us/step) and the step got 3.6% slower
# (profiles/bench_steady_state_wgrad_stream_r1.txt); round 2 at bs512 (GEMM-route
# 1x1 wgrads included): ResNet-18 -4 %, ResNet-50 +0.7 % (noise), and replaying
# the graph on a high-priority stream -30 % (profiles/wgrad_stream_ab_r2.txt).
_WG_STREAM_ENABLED = os.environ.get("DMP_WGRAD_STREAM", "0") == "1"
_WG_STREAMS: dict = {}
_WG_KEEP: list = []          # operands kept alive until the join
_WG_JOIN_QUEUED = [False]


def _wg_join():
    _WG_JOIN_QUEUED[0] = False
    cur = torch.cuda.current_stream()
    for side in _WG_STREAMS.values():
        cur.wait_stream(side)
    _WG_KEEP.clear()


def _side_wgrad(dev, fn, *keep):
    """Run ``fn()`` on the device's wgrad stream (ordered after the current stream)."""
    side = _WG_STREAMS.get(dev)
    if side is None:
        side = _WG_STREAMS[dev] = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        fn()
    _WG_KEEP.append(keep)
    if not _WG_JOIN_QUEUED[0]:
        _WG_JOIN_QUEUED[0] = True
        torch.autograd.Variable._execution_engine.queue_callback(_wg_join)


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


_IGEMM_ROWS_IDS = range(24, 28)   # forward tiles with the row-staged epilogue (csrc/conv.hip)


def _igemm_candidates(out_channels: int, fwd: bool = True):
    return [c[0] for c in _configs() if c[2] <= max(64, out_channels)
            and (fwd or c[0] not in _IGEMM_ROWS_IDS)]


def _wgrad_candidates(K: int, CO: int | None = None):
    """cfg = BNW sel | BP32 << 2 | NS3 << 3 | (min P rows / 512) << 4 | BMW128 << 8
    | XCD << 9 (csrc/conv_wgrad.hip); the 128-channel tiles only when ``CO % 128 == 0``.
    XCD: the tiles of one pixel split dealt to one XCD (profiles/wgrad_xcd_deal_r5.txt)."""
    cands = []
    for xcd in (0, 1):
        for bm in ((0, 1) if CO is not None and CO % 128 == 0 else (0,)):
            for sel, bnw in ((1, 64), (2, 128), (3, 192)):
                if K % bnw:
                    continue
                for bp32 in (0, 1):
                    for ns3 in (0, 1):
                        for chunk in (1, 2, 4, 8):       # x512 rows of P per block
                            cands.append(sel | (bp32 << 2) | (ns3 << 3) | (chunk << 4) | (bm << 8)
                                         | (xcd << 9))
    return cands


_HALO_ENABLED = os.environ.get("DMP_CONV_HALO", "1") != "0"
_WH_BASE = 1000     # csrc/conv_wgrad.hip kWhBase: halo wgrad cfg ids start here


def _halo_candidates(H, W, C, R, S, stride, pad):
    """3x3 / stride-1 halo-tile kernels (csrc/conv.hip conv_halo_kernel) that apply
    to a conv gathering a [*, C, H, W] input; timed by the tuner next to the
    implicit-GEMM tiles."""
    if not _HALO_ENABLED:
        return []
    return list(native().conv_halo_configs(H, W, C, R, S, stride, pad))


# ---------------------------------------------- 1x1 / stride-1 convs as GEMMs
# A 1x1 stride-1 unpadded conv over channels_last NHWC rows IS a GEMM:
#   fwd   Y[m][co] = X[m][:] . W[co][:]     (csrc/gemm.hip mode 0, + BN partial
#                                            sums of the stored outputs)
#   dgrad dX = dY W                         (mode 1, + the shortcut-alias addend)
#   wgrad dW += dY^T X                      (mode 2, fp32 into the arena view)
# The MFMA GEMM reaches 800-1000 TF/s on these shapes where the implicit-GEMM
# conv tiles (built around the tap gather) stay at 500-700
# (profiles/gemm_vs_hipblaslt_r2.txt, linear_vs_conv1x1_r1.txt): the route is a
# tuner candidate (_GEMM_ROUTE) next to the conv tiles for every such layer
# (the ResNet-50 bottleneck's 1x1 convs).
_GEMM_ROUTE = 30000
_GEMM_1X1 = os.environ.get("DMP_CONV_GEMM1X1", "1") != "0"


def _gemm1x1_ok(w_shape, stride, pad, ci, co) -> bool:
    return (_GEMM_1X1 and tuple(w_shape[2:]) == (1, 1) and stride == 1 and pad == 0
            and ci % 8 == 0 and co % 8 == 0)


def _rows_nhwc(t):
    """[B, C, H, W] channels_last -> its [B*H*W, C] row view (no copy)."""
    t = t.contiguous(memory_format=torch.channels_last)
    return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1])


def _gemm1x1_fwd(x, w16, part=None, relu=False):
    from .linear import gemm

    B, CI, H, W = x.shape
    CO = w16.shape[0]
    y2 = torch.empty(B * H * W, CO, dtype=x.dtype, device=x.device)
    gemm(0, 0, _rows_nhwc(x), w16.reshape(CO, CI), y2, relu=relu, part=part)
    return y2.view(B, H, W, CO).permute(0, 3, 1, 2)


def _gemm1x1_dgrad(dy, w16, addend=None, addend_mask=None):
    from .linear import gemm

    B, CO, H, W = dy.shape
    CI = w16.shape[1]
    dx2 = torch.empty(B * H * W, CI, dtype=dy.dtype, device=dy.device)
    aux = _rows_nhwc(addend) if addend is not None else None
    gemm(1, 0, _rows_nhwc(dy), w16.reshape(CO, CI), dx2, aux=aux,
         auxmask=addend_mask if aux is not None else None)
    return dx2.view(B, H, W, CI).permute(0, 3, 1, 2)


def _gemm1x1_wgrad(dy, x, g):
    """g: fp32 [CO, CI, 1, 1] (channels_last) accumulated in place."""
    from .linear import gemm

    gemm(2, 3, _rows_nhwc(dy), _rows_nhwc(x), g.reshape(g.shape[0], g.shape[1]))


# ------------------------------------ weight gradient as patch matrix x GEMM
# dW[co][(r, s, ci)] += sum_p dY[p][co] cols[p][(r, s, ci)]: the native patch
# matrix (csrc/im2col.hip, 16-B taps when CI % 8 == 0) into the wgrad GEMM
# (mode 2, split-K over the pixels, fp32 into the arena view -- the
# channels_last [CO][R][S][CI] gradient IS the [CO][K] GEMM output).  A tuner
# candidate for the small-map layers (ResNet-18 layer3 / layer4 at the
# reference batch 64: 1024-4096 pixels, 256-512 channels), bounded by the patch
# matrix size.  Opt-in (DMP_CONV_IM2COL_WGRAD=1): graph-replayed per-candidate
# timing put it at 2.2-6x the gather / halo picks on every ResNet-18 bs64 3x3
# key (45-61 vs 7-22 us: the patch-matrix write plus a short-K GEMM launch,
# profiles/im2col_wgrad_route_r6.txt), so the tuner is not offered it by default.
_IM2COL_ROUTE = 30001
_IM2COL_WGRAD = os.environ.get("DMP_CONV_IM2COL_WGRAD", "0") == "1"
_IM2COL_WGRAD_MAX_BYTES = 64 << 20


def _im2col_wgrad_ok(x, shape, stride, pad) -> bool:
    CO, CI, R, S = shape
    if not _IM2COL_WGRAD or (R, S) == (1, 1) or CI % 8 or CO % 8:
        return False
    B, _, H, W = x.shape
    OH, OW = (H + 2 * pad - R) // stride + 1, (W + 2 * pad - S) // stride + 1
    return 2 * B * OH * OW * R * S * CI <= _IM2COL_WGRAD_MAX_BYTES


def _im2col_wgrad(dy, x, g, stride, pad):
    """g: fp32 [CO, CI, R, S] channels_last, accumulated in place."""
    from .linear import gemm

    CO, CI, R, S = g.shape
    K = R * S * CI
    cols = native().im2col(x.contiguous(memory_format=torch.channels_last), R, S, stride, pad, K)
    gemm(2, 3, _rows_nhwc(dy), cols, g.permute(0, 2, 3, 1).reshape(CO, K))


def _gemm_route_wgrad(route, dy, x, g, stride, pad):
    if route == _IM2COL_ROUTE:
        _im2col_wgrad(dy, x, g, stride, pad)
    else:
        _gemm1x1_wgrad(dy, x, g)


def _fwd_cfg(x, w16, stride, pad):
    key = ("fwd", *x.shape, w16.shape[0], w16.shape[2], w16.shape[3], stride, pad)
    cands = _igemm_candidates(w16.shape[0]) + _halo_candidates(
        x.shape[2], x.shape[3], x.shape[1], w16.shape[2], w16.shape[3], stride, pad)
    if _gemm1x1_ok(w16.shape, stride, pad, x.shape[1], w16.shape[0]):
        cands.append(_GEMM_ROUTE)

    def run(c):
        if c == _GEMM_ROUTE:
            part = torch.zeros(2 * BN_SLOTS * w16.shape[0] + BN_TAIL, dtype=torch.float32,
                               device=x.device)
            _gemm1x1_fwd(x, w16, part)
        else:
            native().conv_fwd(x, w16, stride, pad, True, c)
    return TUNER.best(key, run, cands)


def _dgrad_cfg(dy, w16, H, W, stride, pad):
    key = ("dgrad", *dy.shape, w16.shape[1], H, W, w16.shape[2], w16.shape[3], stride, pad)
    # the row-staged epilogue tiles apply to stride-1 data gradients too
    cands = _igemm_candidates(w16.shape[1], fwd=stride == 1)
    if (H, W) == tuple(dy.shape[2:]):
        cands += _halo_candidates(H, W, dy.shape[1], w16.shape[2], w16.shape[3], stride, pad)
    elif _HALO_ENABLED and stride == 2:
        # 3x3 / stride-2: parity classes run as halo tiles over dY (conv_dgrad_s2_kernel)
        cands += list(native().conv_dgrad_s2_configs(H, W, dy.shape[2], dy.shape[3], dy.shape[1],
                                                     w16.shape[1], w16.shape[2], w16.shape[3],
                                                     stride, pad))
    if _gemm1x1_ok(w16.shape, stride, pad, w16.shape[1], w16.shape[0]):
        cands.append(_GEMM_ROUTE)

    def run(c):
        if c == _GEMM_ROUTE:
            _gemm1x1_dgrad(dy, w16)
        else:
            native().conv_dgrad(dy, w16, H, W, stride, pad, c)
    return TUNER.best(key, run, cands)


def _wgrad_cfg(dy, x, shape, stride, pad):
    key = ("wgrad", *x.shape, *shape, stride, pad)
    if key in TUNER.cache or not TUNER.enabled:
        return TUNER.cache.get(key, -1)
    scratch = torch.empty(shape, dtype=torch.float32, device=x.device,
                          memory_format=torch.channels_last).zero_()
    K = shape[1] * shape[2] * shape[3]
    cands = _wgrad_candidates(K, shape[0])
    if _HALO_ENABLED:
        cands += list(native().conv_wgrad_halo_configs(x.shape[0], x.shape[2], x.shape[3],
                                                       shape[1], shape[0], shape[2], shape[3],
                                                       stride, pad))
    if _gemm1x1_ok(shape, stride, pad, shape[1], shape[0]):
        cands.append(_GEMM_ROUTE)
    elif _im2col_wgrad_ok(x, shape, stride, pad):
        cands.append(_IM2COL_ROUTE)

    def run(c):
        if c in (_GEMM_ROUTE, _IM2COL_ROUTE):
            _gemm_route_wgrad(c, dy, x, scratch, stride, pad)
        else:
            native().conv_wgrad(dy, x, scratch, stride, pad, c)
    return TUNER.best(key, run, cands)


class _NativeConv(Function):
    @staticmethod
    def forward(ctx, x, w16, master, stride, pad, want_stats, slots=None, bias=None, alias=False,
                relu=False):
        # the BN-partials output never receives a gradient: do not let autograd
        # materialise (zero-fill) one for it every backward
        ctx.set_materialize_grads(False)
        cfg = _fwd_cfg(x, w16, stride, pad)
        b32 = None
        if bias is not None:
            b32 = bias.detach()
            if b32.dtype != torch.float32 or not b32.is_contiguous():
                b32 = b32.float().contiguous()
        ctx.bias = bias
        if cfg == _GEMM_ROUTE and b32 is not None:
            cfg = -1                     # the GEMM store epilogue takes no fp32 conv bias
        if cfg == _GEMM_ROUTE:
            part = None
            if want_stats:
                part = slots if slots is not None else torch.zeros(
                    2 * BN_SLOTS * w16.shape[0] + BN_TAIL, dtype=torch.float32, device=x.device)
            y = _gemm1x1_fwd(x, w16, part, relu)
        else:
            y, part, _ = native().conv_fwd(x, w16, stride, pad, want_stats, cfg, slots, b32,
                                           relu)
        # ReLU fused in the epilogue; its backward masks dY by the saved output
        ctx.save_for_backward(x, w16, y if relu else None)
        # input produced by a training BatchNorm(+ReLU): its backward reduce can
        # run in this conv's dgrad epilogue (ops/functional.py BNLink)
        link = getattr(x, "_dmp_bnlink", None)
        ctx.bnlink = link if link is not None and link.consumer_ok(x) else None
        ctx.master = master
        ctx.geom = (x.shape[2], x.shape[3], stride, pad)
        # alias: x handed back as a third output (a view whose gradient arrives
        # here) -- a block routes its shortcut through it, so the shortcut's
        # gradient is added inside this conv's dgrad epilogue instead of by an
        # autograd add over the whole activation
        # alias == "sub": hand back x[:, :, ::2, ::2] instead -- the input of a 1x1 /
        # stride-2 shortcut, which then runs as a stride-1 GEMM; its gradient lands
        # on the stride-2 dgrad's parity class (0, 0) (this conv has stride 2) or
        # is added onto the strided positions of dX after the dgrad (stride 1)
        ctx.alias_sub = alias == "sub" and x.shape[1] % 8 == 0
        if ctx.alias_sub:
            xa = native().subsample2(x)
        else:
            xa = x if alias else None
        if want_stats:
            ctx.mark_non_differentiable(part)
            return y, part, xa
        return y, None, xa

    @staticmethod
    def backward(ctx, dy, _dpart, dxa=None):
        if dy is None:
            # only the alias output received a gradient: it is x's whole gradient
            dx = None
            if dxa is not None and ctx.needs_input_grad[0]:
                dxa = resolve_deferred(dxa)
                if ctx.alias_sub:
                    x = ctx.saved_tensors[0]
                    dx = torch.zeros(x.shape, dtype=dxa.dtype, device=dxa.device).contiguous(
                        memory_format=torch.channels_last)
                    dx[:, :, ::2, ::2] = dxa
                else:
                    dx = dxa
            return dx, None, None, None, None, None, None, None, None, None
        x, w16, y = ctx.saved_tensors
        H, W, stride, pad = ctx.geom
        masked = is_relu_masked(dy)           # the consumer applied relu'(y) already
        dy = dy.contiguous(memory_format=torch.channels_last)
        if y is not None and not masked:
            dy = native().relu_bwd(dy, y)
        dx = None
        master = ctx.master
        # residual gradient handed over unmasked (ops/functional.py deferred
        # residual mask): the native dgrad epilogue applies the bit mask; every
        # other use of dxa gets the masked tensor
        amask = deferred_mask(dxa)
        if amask is not None and (ctx.alias_sub or not ctx.needs_input_grad[0]):
            dxa, amask = apply_bitmask(dxa, amask), None
        elif amask is not None:
            DEFER_RES_STATS["native"] += 1
        sub = ctx.alias_sub and dxa is not None
        sub_after = None          # subsampled alias gradient added after the dgrad
        if sub and not ctx.needs_input_grad[0]:
            dx = torch.zeros(x.shape, dtype=dxa.dtype, device=dxa.device).contiguous(
                memory_format=torch.channels_last)
            dx[:, :, ::2, ::2] = dxa
            dxa = None
        elif sub and (stride != 2 or _dgrad_cfg(dy, w16, H, W, stride, pad) == _GEMM_ROUTE):
            sub_after, dxa, sub = dxa.contiguous(memory_format=torch.channels_last), None, False
        if ctx.needs_input_grad[0] and _dgrad_cfg(dy, w16, H, W, stride, pad) == _GEMM_ROUTE:
            dx = _gemm1x1_dgrad(dy, w16, dxa, amask)
        elif ctx.needs_input_grad[0]:
            cfg = _dgrad_cfg(dy, w16, H, W, stride, pad)
            wt = None
            ref = getattr(master, "_dmp_arena_ref", None)
            arena = ref() if ref is not None else None
            shadow = getattr(master, "_dmp_w16", None)
            if arena is not None and shadow is not None and shadow.data_ptr() == w16.data_ptr():
                wt = arena.transposed_conv_shadow(master)
            bn = ctx.bnlink
            if bn is not None:
                dx = native().conv_dgrad(dy, w16, H, W, stride, pad, cfg, wt, dxa, bn_x=bn.x,
                                         bn_mask=(x if bn.relu == 1 else
                                                  bn.mask if bn.relu == 3 else None),
                                         bn_stats=bn.stats, bn_part=bn.part, bn_relu=bn.relu,
                                         addend_sub=sub, addend_mask=amask)
                bn.fused = (dx, dx._version)
            else:
                dx = native().conv_dgrad(dy, w16, H, W, stride, pad, cfg, wt, dxa,
                                         addend_sub=sub, addend_mask=amask)
        elif dxa is not None:
            dx = dxa
        if sub_after is not None:
            dx = dx.contiguous(memory_format=torch.channels_last)
            native().add_subsampled2(dx, sub_after)
            link = ctx.bnlink
            if link is not None and link.fused is not None:
                # the native in-place add does not bump autograd's version counter:
                # invalidate the BN partials the fused dgrad epilogue recorded (they
                # miss the added gradient) so the BN backward redoes its reduce
                link.fused = (link.fused[0], -1)
        gw = None
        bias = ctx.bias
        # a conv bias gradient (AlexNet) summed by the gather wgrad kernel from the
        # dY tiles it already stages (no separate column-sum launches)
        bias_in_wgrad = False
        if master is not None and master.requires_grad:
            wcfg = _wgrad_cfg(dy, x, tuple(master.shape), stride, pad)
            g = master.grad if getattr(master, "_dmp_arena", False) else None
            bias_in_wgrad = (bias is not None and bias.requires_grad and wcfg < _WH_BASE
                             and getattr(bias, "_dmp_arena", False)
                             and bias.grad is not None and bias.grad.is_contiguous()
                             and bias.grad.dtype == torch.float32
                             and g is not None and g.is_contiguous(
                                 memory_format=torch.channels_last)
                             and getattr(master, "_dmp_grad_ready", None) is None)
            if wcfg in (_GEMM_ROUTE, _IM2COL_ROUTE):
                gg = g if g is not None and g.is_contiguous(
                    memory_format=torch.channels_last) else None
                if gg is None:
                    gw = torch.zeros(tuple(master.shape), dtype=torch.float32, device=x.device)
                    gw = gw.contiguous(memory_format=torch.channels_last)
                    _gemm_route_wgrad(wcfg, dy, x, gw, stride, pad)
                    gw = gw.to(master.dtype)
                else:
                    cb = getattr(master, "_dmp_grad_ready", None)
                    if cb is None and _WG_STREAM_ENABLED:
                        _side_wgrad(x.device,
                                    lambda: _gemm_route_wgrad(wcfg, dy, x, gg, stride, pad), dy, x)
                    else:
                        _gemm_route_wgrad(wcfg, dy, x, gg, stride, pad)
                        if cb is not None:
                            cb(master)
            elif bias_in_wgrad:
                native().conv_wgrad(dy, x, g, stride, pad, wcfg, bias.grad)
            elif g is not None and g.is_contiguous(memory_format=torch.channels_last):
                cb = getattr(master, "_dmp_grad_ready", None)
                if cb is None and _WG_STREAM_ENABLED:
                    _side_wgrad(x.device, lambda: native().conv_wgrad(dy, x, g, stride, pad, wcfg),
                                dy, x)
                else:
                    native().conv_wgrad(dy, x, g, stride, pad, wcfg)
                    if cb is not None:
                        cb(master)
            else:
                gw = torch.zeros(tuple(master.shape), dtype=torch.float32, device=x.device)
                gw = gw.contiguous(memory_format=torch.channels_last)
                native().conv_wgrad(dy, x, gw, stride, pad, wcfg)
                gw = gw.to(master.dtype)
        gb = None
        if bias is not None and bias.requires_grad and not bias_in_wgrad:
            if (getattr(bias, "_dmp_arena", False) and bias.grad is not None
                    and dy.shape[1] % 8 == 0):
                from .linear import bias_grad_acc

                bias_grad_acc(dy, bias.grad)
                cb = getattr(bias, "_dmp_grad_ready", None)
                if cb is not None:
                    cb(bias)
            else:
                gb = dy.sum(dim=(0, 2, 3), dtype=torch.float32).to(bias.dtype)
        return dx, None, gw, None, None, None, None, gb, None, None


def _ceil8(v: int) -> int:
    return (v + 7) // 8 * 8


class _Im2colConv(Function):
    """Any-geometry conv (few input or output channels, large windows: AlexNet's
    11x11/s4 stem, the LeNet convs, the ResNet-50 7x7 stem) as a native patch
    matrix (csrc/im2col.hip) times the weight on the native MFMA GEMM
    (csrc/gemm.hip): bias / ReLU in the GEMM epilogue, weight (+ bias) gradient
    fp32-accumulated into the arena by the wgrad GEMM, input gradient = dgrad
    GEMM into patch space + gather-form col2im.  The patch matrix is kept for
    the weight gradient (no second im2col)."""

    @staticmethod
    def forward(ctx, x, w16, master, b16, bias, stride, pad, relu):
        from .linear import gemm

        B, CI, H, W = x.shape
        CO, _, R, S = master.shape
        K = R * S * CI
        Kp = _ceil8(K)
        cols = native().im2col(x, R, S, stride, pad, Kp)
        wmat = w16.permute(0, 2, 3, 1).reshape(CO, K)       # channels_last: [CO][R][S][CI]
        wp = wmat
        if Kp != K:
            # the arena's batched padded-row image (one launch per step for every
            # such layer), else a one-off padded copy
            ref = getattr(master, "_dmp_arena_ref", None)
            arena = ref() if ref is not None else None
            shadow = getattr(master, "_dmp_w16", None)
            wp = None
            if arena is not None and shadow is not None and shadow.data_ptr() == w16.data_ptr():
                wp = arena.padded_rows_shadow(master, Kp)
            if wp is None:
                wp = torch.zeros(CO, Kp, dtype=w16.dtype, device=w16.device)
                wp[:, :K] = wmat
        OH = (H + 2 * pad - R) // stride + 1
        OW = (W + 2 * pad - S) // stride + 1
        y2 = torch.empty(B * OH * OW, CO, dtype=x.dtype, device=x.device)
        gemm(0, 0, cols, wp, y2, bias=b16, relu=relu)
        ctx.save_for_backward(cols, wp, y2 if relu else None)
        ctx.params = (master, bias)
        ctx.geom = (B, CI, H, W, R, S, K, stride, pad)
        return y2.view(B, OH, OW, CO).permute(0, 3, 1, 2)     # channels_last NCHW view

    @staticmethod
    def backward(ctx, dy):
        from .linear import _arena_grad, gemm
        from .functional import _notify

        cols, wp, y2 = ctx.saved_tensors
        master, bias = ctx.params
        B, CI, H, W, R, S, K, stride, pad = ctx.geom
        CO = master.shape[0]
        masked = is_relu_masked(dy)
        dy2 = dy.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1).reshape(-1, CO)
        if y2 is not None and not masked:
            dy2 = native().relu_bwd(dy2, y2)
        gw = gb = None
        wants_w = master is not None and master.requires_grad
        wants_b = bias is not None and bias.requires_grad
        g = _arena_grad(master) if wants_w else None
        gbias = _arena_grad(bias) if wants_b else None
        tmp_w = wants_w and g is None
        tmp_b = wants_b and gbias is None
        if wants_w or wants_b:
            gmat = (torch.zeros(CO, K, dtype=torch.float32, device=dy.device) if g is None
                    else g)                                   # [CO, K] view of the arena grad
            if tmp_b:
                gbias = torch.zeros(CO, dtype=torch.float32, device=dy.device)
            gemm(2, 3, dy2, cols[:, :K], gmat, dbias=gbias)
            if tmp_w:
                gw = gmat.view(CO, R, S, CI).permute(0, 3, 1, 2).to(master.dtype)
            elif wants_w:
                _notify(master)
            if tmp_b:
                gb = gbias.to(bias.dtype)
            elif wants_b:
                _notify(bias)
        dx = None
        if ctx.needs_input_grad[0]:
            dcols = torch.empty(dy2.shape[0], wp.shape[1], dtype=dy2.dtype, device=dy2.device)
            gemm(1, 0, dy2, wp, dcols)
            dx = native().col2im(dcols, B, CI, H, W, R, S, stride, pad)
        return dx, None, gw, None, gb, None, None, None


class _SmallConv(Function):
    """Stem conv: forward + weight gradient only (the input is data)."""

    @staticmethod
    def forward(ctx, x, w16, master, stride, pad, want_stats, slots=None):
        ctx.set_materialize_grads(False)
        y, part, _ = native().conv_small_fwd(x, w16, stride, pad, want_stats, slots)
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
            return None, None, None, None, None, None, None
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
        return None, None, gw, None, None, None, None


class _StemConv(Function):
    """ImageNet 7x7/2/3 stem (3 -> 64 channels, csrc/stem.hip): the input is
    space-to-depth packed once (2x2 pixel blocks -> 16 channels, the 4th colour
    channel zero) so the conv becomes a stride-1 4x4 conv with K = 256 on MFMA;
    the forward folds the BN partial sums into its store epilogue, the weight
    gradient runs in the packed space and is folded back into the 7x7 arena
    gradient.  The packed input is kept for the weight gradient (the stem's
    input is data: no input gradient)."""

    @staticmethod
    def forward(ctx, x, w16, master, want_stats, slots=None):
        ctx.set_materialize_grads(False)
        y, part, xs = native().stem_fwd(x, w16, want_stats, slots)
        ctx.save_for_backward(xs)
        ctx.master = master
        if want_stats:
            ctx.mark_non_differentiable(part)
            return y, part
        return y, None

    @staticmethod
    def backward(ctx, dy, _dpart):
        if dy is None:
            return None, None, None, None, None
        (xs,) = ctx.saved_tensors
        master = ctx.master
        gw = None
        if master is not None and master.requires_grad:
            g = master.grad if getattr(master, "_dmp_arena", False) else None
            if g is not None and g.is_contiguous(memory_format=torch.channels_last):
                native().stem_wgrad(dy, xs, g)
                cb = getattr(master, "_dmp_grad_ready", None)
                if cb is not None:
                    cb(master)
            else:
                gw = torch.empty(tuple(master.shape), dtype=torch.float32, device=xs.device,
                                 memory_format=torch.channels_last).zero_()
                native().stem_wgrad(dy, xs, gw)
                gw = gw.to(master.dtype)
        return None, None, gw, None, None


def stem_conv_supported(x, weight, stride, padding, dilation, groups) -> bool:
    if not (_NATIVE_ENABLED and _STEM != "im2col" and x.is_cuda and x.dtype == torch.bfloat16
            and x.dim() == 4):
        return False
    if x.requires_grad or groups != 1 or _pair(dilation) != (1, 1):
        return False
    if _pair(stride) != (2, 2) or _pair(padding) != (3, 3):
        return False
    if tuple(weight.shape) != (64, 3, 7, 7):
        return False
    return bool(native().stem_supported(x.shape[2], x.shape[3]))


def small_conv_supported(x, weight, stride, padding, dilation, groups) -> bool:
    if not (_NATIVE_ENABLED and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4):
        return False
    if x.requires_grad or groups != 1 or _pair(dilation) != (1, 1):
        return False
    st, pd = _pair(stride), _pair(padding)
    if st[0] != st[1] or pd[0] != pd[1] or not isinstance(pd[0], int):
        return False
    co, ci, r, s = weight.shape
    # VALU kernels: the pick only while K = R*S*CI is tiny (CIFAR-style 3x3x3
    # stems); the 7x7 stem runs on csrc/stem.hip, 11x11 / 5x5 on im2col + GEMM
    return co % 64 == 0 and r * s * ci <= _SMALL_MAX_K


BN_SLOTS = 64   # csrc/bn_slots.h kBnSlots
BN_TAIL = 4     # csrc/bn_slots.h kBnTail (arrival ticket)


def bn_slot_buffer(owner, attr: str, channels: int, device, fresh: bool = True):
    """Persistent zeroed ``[2][BN_SLOTS][channels] + BN_TAIL`` fp32 slot buffer on ``owner``.

    ``fresh``: the caller is about to accumulate into it, so sums a folded BN
    forward left behind without a matching backward (``mark_slots``, see
    ``ops.functional._BNAct``) are zeroed first."""
    n = 2 * BN_SLOTS * channels + BN_TAIL
    buf = getattr(owner, attr, None)
    if buf is None or buf.device != device or buf.numel() != n:
        buf = torch.zeros(n, dtype=torch.float32, device=device)
        object.__setattr__(owner, attr, buf)
    elif fresh:
        from .functional import clean_slots

        clean_slots(buf)
    return buf


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


def im2col_conv_supported(x, weight, stride, padding, dilation, groups) -> bool:
    """Any other conv with a bf16 GPU input: patch matrix + native GEMM."""
    if not (_NATIVE_ENABLED and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4):
        return False
    if groups != 1 or _pair(dilation) != (1, 1):
        return False
    st, pd = _pair(stride), _pair(padding)
    return st[0] == st[1] and pd[0] == pd[1] and isinstance(pd[0], int)


def conv2d(x, w, b, stride, padding, dilation, groups, master=None, want_stats=False,
           slots=None, alias=False, relu=False):
    """Returns ``y`` (with BN slot sums attached as ``y._dmp_bn_part`` when ``want_stats``).

    ``slots``: the layer's persistent ``[2][64][CO]`` fp32 BN slot buffer (zeroed;
    the consuming BatchNorm's finalize re-zeroes it); a fresh one when None.
    ``alias``: return ``(y, x_alias)``; gradients reaching ``x_alias`` are summed
    into this conv's input gradient by the dgrad kernel itself.  ``alias="sub"``
    (native stride-2 convs): ``x_alias`` is ``x[:, :, ::2, ::2]`` (gathered), the
    input of a 1x1 / stride-2 shortcut run at stride 1; other routes hand back x.
    """
    if x.is_cuda and x.dim() == 4:
        x = x.contiguous(memory_format=torch.channels_last)
        if master is not None and native_conv_supported(
                x, master, stride, padding, dilation, groups):
            w16 = getattr(master, "_dmp_w16", None)
            if w16 is None or not w16.is_contiguous(memory_format=torch.channels_last):
                w16 = master.detach().to(torch.bfloat16).contiguous(
                    memory_format=torch.channels_last)
            y, part, xa = _NativeConv.apply(x, w16, master, _pair(stride)[0], _pair(padding)[0],
                                            bool(want_stats and not relu),
                                            slots if want_stats and not relu else None, b,
                                            alias if alias == "sub" else bool(alias),
                                            bool(relu))
            if xa is not None:
                # (the object apply() returned: x handed back is a new view of x)
                xa._dmp_conv_alias = True   # its gradient may carry a deferred mask
            if part is not None:
                y._dmp_bn_part = part
            set_nonneg(y, relu)
            return (y, xa) if alias else y
        if master is not None and b is None and not relu and _STEM != "im2col" and \
                small_conv_supported(x, master, stride, padding, dilation, groups):
            w16 = getattr(master, "_dmp_w16", None)
            if w16 is None or not w16.is_contiguous(memory_format=torch.channels_last):
                w16 = master.detach().to(torch.bfloat16).contiguous(
                    memory_format=torch.channels_last)
            y, part = _SmallConv.apply(x, w16, master, _pair(stride)[0], _pair(padding)[0],
                                       bool(want_stats), slots if want_stats else None)
            if part is not None:
                y._dmp_bn_part = part
            return (y, x) if alias else y
        if master is not None and b is None and not relu and \
                stem_conv_supported(x, master, stride, padding, dilation, groups):
            w16 = getattr(master, "_dmp_w16", None)
            if w16 is None or not w16.is_contiguous(memory_format=torch.channels_last):
                w16 = master.detach().to(torch.bfloat16).contiguous(
                    memory_format=torch.channels_last)
            y, part = _StemConv.apply(x, w16, master, bool(want_stats),
                                      slots if want_stats else None)
            if part is not None:
                y._dmp_bn_part = part
            return (y, x) if alias else y
        if master is not None and im2col_conv_supported(x, master, stride, padding, dilation,
                                                        groups):
            w16 = getattr(master, "_dmp_w16", None)
            if w16 is None or not w16.is_contiguous(memory_format=torch.channels_last):
                w16 = master.detach().to(torch.bfloat16).contiguous(
                    memory_format=torch.channels_last)
            b16 = None
            if b is not None:
                b16 = getattr(b, "_dmp_w16", None)
                if b16 is None:
                    b16 = b.detach().to(torch.bfloat16).contiguous()
            y = _Im2colConv.apply(x, w16, master, b16, b, _pair(stride)[0], _pair(padding)[0],
                                  bool(relu))
            set_nonneg(y, relu)
            return (y, x) if alias else y
        if w is None:
            w = master.to(x.dtype)
    stock_gpu("conv2d", x, reason=f"input {tuple(x.shape)} {x.dtype}, weight "
              f"{tuple((w if w is not None else master).shape)}, stride {stride}, padding "
              f"{padding}, groups {groups}")
    y = F.conv2d(x, w, b if b is None or b.dtype == x.dtype else b.to(x.dtype), stride, padding,
                 dilation, groups)
    if relu:
        y = F.relu(y)
    return (y, x) if alias else y
