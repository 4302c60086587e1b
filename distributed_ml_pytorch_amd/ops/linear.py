"""Fully-connected layers on the native MFMA GEMM (``csrc/gemm.hip``).

Parity: the reference's ``nn.Linear`` layers (/root/reference/example/models.py:
11-13 LeNet fc1-3, :43 AlexNet classifier; ATen ``addmm`` / ``mm`` / ``sum`` rows
of SURVEY §2.3) in fp32; here bf16 compute with fp32 master weights.

All three passes of a linear layer run on one hand-written gfx950 kernel family:

* forward ``Y = X W^T + b``: bias folded into the accumulator init; the ViT MLP
  runs fc1 with a GELU epilogue that writes both the pre-activation ``h`` (kept
  for backward) and ``gelu(h)`` (fc2's input) -- no separate GELU pass;
* data gradient ``dX = dY W``: W is read k-strided through transposed LDS reads
  (no transposed weight copy); in the MLP the fc2 dgrad epilogue multiplies by
  ``gelu'(h)`` so it produces fc1's output gradient directly;
* weight gradient ``dW += dY^T X``: fp32 accumulated straight into the flat
  grad arena (split-K with atomics when the output is small), the bias
  gradient summed by the same kernel from the dY tiles it already stages.

Tile shape (and split-K) are picked per (pass, shape) by measurement on first
use (``ops.tuner``); shapes the 16-B DMA tiles cannot take (a dimension not a
multiple of 8: 10-class heads, LeNet's 84-wide layer) run the any-shape
fallback kernel of the same file.  No library GEMM is ever a candidate: every
Linear pass of every model runs on these kernels (round 6 took the hipBLASLt
candidate of round 5 back out; the QKV forward it won is tracked
in profiles/gemm_native_only_r6.txt).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F
from torch.autograd import Function

from ._ext import native
from .functional import _notify, is_relu_masked, mark_relu_masked, nonneg, set_nonneg
from .tuner import TUNER

_SMALL = -1            # any-shape fallback kernel


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


# ----------------------------------------------------------------- dispatcher
def _mfma_ok(mode: int, M: int, N: int, K: int, *mats) -> bool:
    """The MFMA tiles' layout constraints (mirrors the checks in bindings.cpp)."""
    for t in mats:
        if t is None:
            continue
        if t.stride(-1) != 1 or t.data_ptr() % 16 or (t.shape[0] > 1 and t.stride(0) % 8):
            return False
    a, b = mats[0], mats[1]
    c8 = lambda v: (v + 7) // 8 * 8                      # noqa: E731
    if mode == 0:
        return K % 8 == 0
    if mode == 1:
        return K % 8 == 0 and (N % 8 == 0 or b.stride(0) >= c8(N))
    return ((M % 8 == 0 or a.stride(0) >= c8(M))          # pieces may run into row padding
            and (N % 8 == 0 or b.stride(0) >= c8(N)))


# candidate encoding: (cfg + 1) * 1024 + splits (cfg -1 = any-shape kernel),
# + _SLAB for a wgrad split-K reduced through a plain-store slab instead of fp32
# atomics; the tuner's "no pick" is -1
_SLAB = 1 << 20


def _enc(cfg: int, splits: int, slab: bool = False) -> int:
    return (cfg + 1) * 1024 + splits + (_SLAB if slab else 0)


def _dec(e: int):
    return (e % _SLAB) // 1024 - 1, e % 1024


def _dec_slab(e: int) -> bool:
    return e >= _SLAB


def _wgrad_splits(M: int, N: int, K: int, bm: int, bn: int):
    """Split-K counts worth timing for an fp32-accumulating weight gradient:
    enough blocks to fill the chip (a conv stem's 64 x 147 output over 1.6M
    pixels is 2 tiles), at least 256 reduction rows per split."""
    tiles = -(-M // bm) * -(-N // bn)
    out = []
    for s in (1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64, 96, 128, 192, 256, 384, 512):
        if s > 1 and K < 256 * s:
            break
        if s == 1 or tiles * s <= 2048:
            out.append(s)
    # keep the few counts around "one block per CU" plus the unsplit one
    if len(out) > 6:
        best = min(out, key=lambda s: abs(tiles * s - 384))
        i = out.index(best)
        out = sorted({1, *out[max(0, i - 2):i + 3]})
    return out


# opt-in (DMP_GEMM_SK=1): measured slower than the unsplit tiles on every ViT-B/16
# fwd / dgrad shape -- the pieces' fp32 publish + combine costs more than the
# partial round it recovers (profiles/gemm_remainder_splitk_r5.txt)
_SK_SPLITS = (2, 4) if os.environ.get("DMP_GEMM_SK", "0") == "1" else ()


def _sk_splits(cfg: int, M: int, N: int, K: int, s: int) -> bool:
    """The fwd / dgrad remainder split-K plan of ``cfg`` splits at ``s``."""
    return native().gemm_sk_pieces(cfg, M, N, K, s) > 0


def _small_splits(mode: int, K: int) -> int:
    """Split-K of the any-shape kernel in wgrad mode: its blocks cover only a
    64x64 output tile, so a long reduction (a conv's B*OH*OW pixels) must be
    spread over blocks (fp32 atomics), ~256 rows each."""
    return max(1, min(1023, K // 256)) if mode == 2 else 1


def _small_split_options(mode: int, K: int):
    """Split-K counts of the any-shape kernel worth timing in wgrad mode: the
    default (~256 rows per split) and finer ones.  A classifier head's weight
    gradient (10 x 512 over a batch of 512) is 8 output tiles; with 2 splits its
    16 blocks walk 8 serial k-stages each and the launch is latency-bound
    (52 us per ResNet-18 step); 16-64 splits finish in one or two stages."""
    if mode != 2:
        return [1]
    return sorted({_small_splits(mode, K)} |
                  {max(1, min(1023, K // r)) for r in (32, 64, 128)})


def _candidates(mode: int, epi: int, M: int, N: int, K: int, ok: bool):
    if not ok:
        return [_enc(_SMALL, s) for s in _small_split_options(mode, K)]
    cands = []
    for c in native().gemm_configs():
        cid, bm, bn = c[0], c[1], c[2]
        if not native().gemm_config_ok(mode, cid):
            continue
        if mode == 2:
            cands += [_enc(cid, s) for s in _wgrad_splits(M, N, K, bm, bn)]
            cands += [_enc(cid, s, True) for s in _wgrad_splits(M, N, K, bm, bn) if s > 1]
        else:
            cands.append(_enc(cid, 1))
            # remainder split-K (csrc/gemm.hip GemmArgs sk_*): the tiles of a last,
            # partial round in k-pieces -- only where the plan actually splits
            cands += [_enc(cid, s) for s in _SK_SPLITS if _sk_splits(cid, M, N, K, s)]
    if M * N * K < (1 << 22):
        cands += [_enc(_SMALL, s) for s in _small_split_options(mode, K)]
    return cands


def _default(mode: int, M: int, N: int, K: int, ok: bool) -> int:
    """Heuristic pick when tuning is off or a graph is being captured."""
    if not ok:
        return _enc(_SMALL, _small_splits(mode, K))
    if mode == 2:
        return _enc(4, _wgrad_splits(M, N, K, 128, 128)[-1])
    return _enc(4, 1)


def gemm(mode: int, epi: int, a, b, c, c2=None, bias=None, aux=None, dbias=None, relu=False,
         part=None, auxmask=None):
    """C = epilogue(A(m,k) B(n,k)) on the native kernels (see csrc/gemm.hip):
    mode 0 fwd (a [M,K], b [N,K]), 1 dgrad (a [M,K], b [K,N]), 2 wgrad (a [K,M],
    b [K,N], fp32 c accumulated); epi 0 store(+bias,+aux), 1 GELU, 2 x gelu'(aux),
    3 fp32 accumulate (+dbias).  ``part``: BatchNorm slot sums [2][64][N] of the
    stored outputs (epi 0, MFMA tiles; a 1x1 conv feeding a BatchNorm).
    ``auxmask``: 1-bit mask of ``aux`` ([M * N / 8] uint8, bn.hip's ReLU mask
    layout) applied by the epilogue; materialised first where the picked kernel
    takes none (any-shape fallback, strided output)."""
    M, N = c.shape
    K = a.shape[0] if mode == 2 else a.shape[1]
    if M == 0 or N == 0:
        return
    # outputs / aux of any row stride: the epilogues fall back to element access
    ok = _mfma_ok(mode, M, N, K, a, b)
    key = ("gemm", mode, epi, M, N, K, bias is not None, aux is not None, dbias is not None,
           bool(relu)) + (("stats",) if part is not None else ())
    pick = TUNER.cache.get(key)
    if pick is None:
        cands = _candidates(mode, epi, M, N, K, ok)
        if part is not None:
            if not ok:
                raise ValueError("gemm: BN partial sums need MFMA-compatible operands")
            cands = [e for e in cands if _dec(e)[0] >= 0]
        if len(cands) == 1:
            pick = cands[0]
        else:
            if mode == 2:      # never time into the live grad arena
                cs = torch.zeros_like(c)
                ds = torch.zeros_like(dbias) if dbias is not None else None
            else:
                cs, ds = c, dbias

            def run(e):
                cfg_e, split_e = _dec(e)
                ps = torch.zeros_like(part) if part is not None else None
                native().gemm(mode, epi, cfg_e, a, b, cs, c2, bias, aux, ds, split_e, relu,
                              ps, _dec_slab(e))
            pick = TUNER.best(key, run, cands)
            if pick == -1:
                pick = _default(mode, M, N, K, ok)
    if auxmask is not None and (_dec(pick)[0] < 0 or epi != 0 or c.stride(0) != N or N % 8):
        from .functional import apply_bitmask_rows

        aux, auxmask = apply_bitmask_rows(aux, auxmask), None
    if pick < 0:
        raise RuntimeError(f"gemm: tune cache entry {pick} for {key} is not a native kernel "
                           "(library GEMMs are not candidates)")
    cfg, splits = _dec(pick)
    native().gemm(mode, epi, cfg, a, b, c, c2, bias, aux, dbias, splits, relu, part,
                  _dec_slab(pick), auxmask)


def _rows(t, k):
    """[.., k] -> a [rows, k] operand with unit inner stride (copies only if needed)."""
    t2 = t.reshape(-1, k)
    if t2.stride(-1) != 1 or t2.data_ptr() % 16 or (t2.shape[0] > 1 and t2.stride(0) % 8):
        t2 = t2.contiguous()
    return t2


# ------------------------------------------------------------ arena plumbing
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


def _weight_grads(dy2, x2, w, b):
    """dW (+ db) of ``y = x W^T + b``: accumulated into the fp32 arena views
    when the parameters live in one (grad-ready hooks fired), else returned."""
    N, K = dy2.shape[1], x2.shape[1]
    gw = gb = None
    g = _arena_grad(w) if w is not None and w.requires_grad else None
    gbias = _arena_grad(b) if b is not None and b.requires_grad else None
    tmp_w = g is None and w is not None and w.requires_grad
    tmp_b = gbias is None and b is not None and b.requires_grad
    if g is None and (tmp_w or tmp_b or gbias is not None):
        g = torch.zeros(N, K, dtype=torch.float32, device=dy2.device)
    if tmp_b:
        gbias = torch.zeros(N, dtype=torch.float32, device=dy2.device)
    if g is not None:
        gemm(2, 3, dy2, x2, g, dbias=gbias)
    if tmp_w:
        gw = g.to(w.dtype)
        if w.dim() == 4:                     # patch embedding: (kh, kw, Cin) columns
            gw = gw.view(w.shape[0], w.shape[2], w.shape[3], w.shape[1]).permute(0, 3, 1, 2)
    elif w is not None and w.requires_grad:
        _notify(w)
    if tmp_b:
        gb = gbias.to(b.dtype)
    elif b is not None and b.requires_grad:
        _notify(b)
    return gw, gb


class _ArenaLinear(Function):
    @staticmethod
    def forward(ctx, x, w16, b16, w, b, relu=False):
        N, K = w16.shape
        x2 = _rows(x, K)
        y = torch.empty(x2.shape[0], N, dtype=x.dtype, device=x.device)
        gemm(0, 0, x2, w16, y, bias=b16, relu=relu)      # ReLU fused in the epilogue
        ctx.save_for_backward(x2, w16, y if relu else None)
        ctx.params = (w, b)
        ctx.xshape = x.shape
        # the input is a ReLU output (or a dropout of one): the data gradient's
        # epilogue applies that ReLU's derivative (EPI_DRELU, mask = input > 0)
        ctx.x_nonneg = nonneg(x)
        return y.view(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, w16, y = ctx.saved_tensors
        w, b = ctx.params
        N, K = w16.shape
        masked = is_relu_masked(dy)
        dy2 = _rows(dy, N)
        if y is not None and not masked:
            dy2 = native().relu_bwd(dy2, y)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(dy2.shape[0], K, dtype=dy.dtype, device=dy.device)
            if ctx.x_nonneg:
                gemm(1, 4, dy2, w16, dx, aux=x2)
            else:
                gemm(1, 0, dy2, w16, dx)
            dx = dx.view(ctx.xshape)
            if ctx.x_nonneg:
                mark_relu_masked(dx)
        gw, gb = _weight_grads(dy2, x2, w, b)
        return dx, None, None, gw, gb, None


# ------------------------------------------------ fused GAP + Linear head
_FUSED_HEAD = os.environ.get("DMP_FUSED_HEAD", "1") != "0"


class _GapLinear(Function):
    """``linear(global_avg_pool(x))`` in one native launch per direction
    (csrc/head.hip): pooled features are kept (bf16) for the weight gradient;
    dW / db accumulate into the fp32 arena like :class:`_ArenaLinear`."""

    @staticmethod
    def forward(ctx, x, w16, b16, w, b):
        y, f = native().gap_linear_fwd(x, w16, b16)
        ctx.save_for_backward(f, w16)
        ctx.params = (w, b)
        ctx.hw = (x.shape[2], x.shape[3])
        return y

    @staticmethod
    def backward(ctx, dy):
        f, w16 = ctx.saved_tensors
        w, b = ctx.params
        N, C = w16.shape
        gw = _arena_grad(w) if w.requires_grad else None
        gb = _arena_grad(b) if b is not None and b.requires_grad else None
        tmp_w = gw is None
        tmp_b = gb is None and b is not None and b.requires_grad
        if tmp_w:
            gw = torch.zeros(N, C, dtype=torch.float32, device=dy.device)
        if tmp_b:
            gb = torch.zeros(N, dtype=torch.float32, device=dy.device)
        dx = native().gap_linear_bwd(dy, f, w16, gw, gb, ctx.hw[0], ctx.hw[1])
        gw_out = gb_out = None
        if w.requires_grad:
            if tmp_w:
                gw_out = gw.to(w.dtype)
            else:
                _notify(w)
        if b is not None and b.requires_grad:
            if tmp_b:
                gb_out = gb.to(b.dtype)
            else:
                _notify(b)
        return dx, None, None, gw_out, gb_out


def gap_linear_ok(x, linear) -> bool:
    """The fused head applies: bf16 channels-last activations, arena-backed
    weights with a bf16 shadow, C % 8 == 0, at most 16 classes."""
    if not (_FUSED_HEAD and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4):
        return False
    if not x.is_contiguous(memory_format=torch.channels_last):
        return False
    w, b = linear.weight, linear.bias
    w16 = getattr(w, "_dmp_w16", None)
    if w16 is None or w16.dtype != x.dtype or not w16.is_contiguous():
        return False
    if b is not None and getattr(b, "_dmp_w16", None) is None:
        return False
    return bool(native().gap_linear_supported(x.shape[1], w.shape[0]))


def gap_linear(x, linear):
    w, b = linear.weight, linear.bias
    b16 = b._dmp_w16 if b is not None else None
    if not _needs_graph(x, w, b):
        return native().gap_linear_fwd(x, w._dmp_w16, b16)[0]
    return _GapLinear.apply(x, w._dmp_w16, b16, w, b)


def arena_linear_ok(x, w, b) -> bool:
    """The weight (and bias) live in an arena with a bf16 shadow matching ``x``
    (training or inference: under ``torch.no_grad()`` the forward runs the same
    native GEMM on the shadow, without an autograd node)."""
    if not (x.is_cuda and x.dtype == torch.bfloat16):
        return False
    w16 = getattr(w, "_dmp_w16", None)
    if w16 is None or w16.dtype != x.dtype or not w16.is_contiguous():
        return False
    return b is None or getattr(b, "_dmp_w16", None) is not None


def _infer_linear(x, w16, b16, relu=False):
    """Forward-only ``x W^T + b`` on the native GEMM (no autograd node, no saved
    tensors): the eval / inference path of every arena-backed Linear (the
    reference evaluates the whole test set every log interval,
    /root/reference/example/main.py:83-84,110-125)."""
    N, K = w16.shape
    x2 = _rows(x, K)
    y = torch.empty(x2.shape[0], N, dtype=x.dtype, device=x.device)
    gemm(0, 0, x2, w16, y, bias=b16, relu=relu)
    return y.view(*x.shape[:-1], N)


def _needs_graph(x, *params) -> bool:
    return torch.is_grad_enabled() and (
        x.requires_grad or any(p is not None and p.requires_grad for p in params))


def linear(x, w, b, relu: bool = False):
    w16 = w._dmp_w16
    b16 = b._dmp_w16 if b is not None else None
    if not _needs_graph(x, w, b):
        return set_nonneg(_infer_linear(x, w16, b16, bool(relu)), relu)
    return set_nonneg(_ArenaLinear.apply(x, w16, b16, w, b, bool(relu)), relu)


# ------------------------------------------------------------ fused ViT MLP
class _ArenaMLP(Function):
    """``fc2(gelu_tanh(fc1(x)))`` as 4 + 1 native GEMMs with the GELU in the
    epilogues: fc1 forward writes (h, gelu(h)); fc2's data gradient multiplies
    by gelu'(h) and IS fc1's output gradient.  Replaces two library GEMMs + a
    GELU pass forward and a GELU-backward pass."""

    @staticmethod
    def forward(ctx, x, w1_16, b1_16, w2_16, b2_16, w1, b1, w2, b2):
        H, D = w1_16.shape
        x2 = _rows(x, D)
        M = x2.shape[0]
        h = torch.empty(M, H, dtype=x.dtype, device=x.device)
        g = torch.empty_like(h)
        gemm(0, 1, x2, w1_16, h, c2=g, bias=b1_16)
        y = torch.empty(M, w2_16.shape[0], dtype=x.dtype, device=x.device)
        gemm(0, 0, g, w2_16, y, bias=b2_16)
        ctx.save_for_backward(x2, h, g, w1_16, w2_16)
        ctx.params = (w1, b1, w2, b2)
        ctx.xshape = x.shape
        return y.view(*x.shape[:-1], y.shape[1])

    @staticmethod
    def backward(ctx, dy):
        x2, h, g, w1_16, w2_16 = ctx.saved_tensors
        w1, b1, w2, b2 = ctx.params
        dy2 = _rows(dy, w2_16.shape[0])
        gw2, gb2 = _weight_grads(dy2, g, w2, b2)
        dh = torch.empty_like(h)
        gemm(1, 2, dy2, w2_16, dh, aux=h)          # (dY W2) * gelu'(h)
        gw1, gb1 = _weight_grads(dh, x2, w1, b1)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x2)
            gemm(1, 0, dh, w1_16, dx)
            dx = dx.view(ctx.xshape)
        return dx, None, None, None, None, gw1, gb1, gw2, gb2


def mlp_ok(x, fc1, fc2) -> bool:
    return (arena_linear_ok(x, fc1.weight, fc1.bias)
            and arena_linear_ok(x, fc2.weight, fc2.bias))


def mlp(x, fc1, fc2):
    """``fc2(gelu_tanh(fc1(x)))`` for two arena-backed linear layers."""
    w1, b1, w2, b2 = fc1.weight, fc1.bias, fc2.weight, fc2.bias
    if not _needs_graph(x, w1, b1, w2, b2):
        # inference: fc1 with the GELU epilogue (h is written but not kept), fc2
        H, D = w1._dmp_w16.shape
        x2 = _rows(x, D)
        h = torch.empty(x2.shape[0], H, dtype=x.dtype, device=x.device)
        g = torch.empty_like(h)
        gemm(0, 1, x2, w1._dmp_w16, h, c2=g, bias=b1._dmp_w16 if b1 is not None else None)
        del h
        return _infer_linear(g, w2._dmp_w16, b2._dmp_w16 if b2 is not None else None).view(
            *x.shape[:-1], w2.shape[0])
    return _ArenaMLP.apply(x, w1._dmp_w16, b1._dmp_w16 if b1 is not None else None,
                           w2._dmp_w16, b2._dmp_w16 if b2 is not None else None, w1, b1, w2, b2)


# ---------------------------------------------------------- patch embedding
def patch_embed_ok(x, w, b, patch: int) -> bool:
    """Non-overlapping ``patch`` x ``patch`` conv whose weight lives in an arena
    with a channels-last bf16 shadow: computable as one GEMM on patch rows."""
    if not (x.is_cuda and x.dtype == torch.bfloat16 and not x.requires_grad
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
    lands in the arena like any linear layer's.  No input gradient (pixels), so
    no dgrad GEMM.  Replaces a library conv forward + backward-weights pair."""
    B, C, H, W = x.shape
    gh, gw = H // patch, W // patch
    K = patch * patch * C
    if K % 8 == 0:
        # native patch rows (csrc/im2col.hip: stride = window, k = (kh, kw, Cin))
        xp = native().im2col(x.contiguous(memory_format=torch.channels_last), patch, patch,
                             patch, 0, K).view(B, gh * gw, K)
    else:
        xp = (x.reshape(B, C, gh, patch, gw, patch).permute(0, 2, 4, 3, 5, 1)
              .reshape(B, gh * gw, K))
    w16 = w._dmp_w16.permute(0, 2, 3, 1).reshape(w.shape[0], -1)
    b16 = b._dmp_w16 if b is not None else None
    if not _needs_graph(x, w, b):
        return _infer_linear(xp, w16, b16)
    return _ArenaLinear.apply(xp, w16, b16, w, b)


def plain_linear(x, w, b):
    """Library fallback (CPU, fp32, no arena)."""
    return F.linear(x, w, b)
