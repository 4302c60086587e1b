"""Flat parameter arena: every parameter and gradient is a view into one buffer.

The reference ravels the model with a ``torch.cat`` over all parameters on
EVERY optimizer step (``ravel_model_params`` at
/root/reference/asgd/optim/Asynchronous.py:27,34,54) and copies slices back on
every pull (``unravel_model_params`` :18).  Here the flat buffer IS the
storage, so ravel/unravel are zero-copy and the ASGD update, the push, the
pull landing and the sync-DP all-reduce each touch one contiguous buffer.

Layout (fp32 master ``p32``, fp32 ``g32`` grads, optional bf16 ``w16`` compute
shadow refreshed by the fused optimizer kernel):
  * parameter order = ``model.parameters()`` order (the reference's ravel order)
  * each parameter starts on a 64-element (256 B) boundary -> every view is
    16-B aligned for the vectorised kernels
  * 4-D weights get channels_last strides (physical [Cout][kh][kw][Cin]), the
    layout the NHWC conv kernels and MIOpen's NHWC path consume
  * the total is padded to a multiple of ``pad_multiple`` elements so the buffer
    splits evenly into world-size shards for reduce-scatter / all-gather.
"""
from __future__ import annotations

from dataclasses import dataclass

import weakref

import torch

ALIGN = 64


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def _strided_view(flat: torch.Tensor, offset: int, like: torch.Tensor, channels_last: bool):
    shape = tuple(like.shape)
    if channels_last and len(shape) == 4:
        n, c, h, w = shape
        stride = (h * w * c, 1, w * c, c)
    else:
        stride = []
        acc = 1
        for s in reversed(shape):
            stride.append(acc)
            acc *= s
        stride = tuple(reversed(stride))
    return torch.as_strided(flat, shape, stride, flat.storage_offset() + offset)


@dataclass
class Slot:
    index: int
    offset: int
    numel: int
    shape: tuple


class FlatArena:
    def __init__(self, params, device=None, shadow_dtype: torch.dtype | None = torch.bfloat16,
                 channels_last: bool = True, pad_multiple: int = ALIGN * 840,
                 with_grads: bool = True):
        if isinstance(params, torch.nn.Module):
            params = list(params.parameters())
        self.params = list(params)
        if not self.params:
            raise ValueError("FlatArena needs at least one parameter")
        dev = torch.device(device) if device is not None else self.params[0].device
        self.device = dev
        self.channels_last = channels_last
        off = 0
        self.slots: list[Slot] = []
        for i, p in enumerate(self.params):
            self.slots.append(Slot(i, off, p.numel(), tuple(p.shape)))
            off = _round_up(off + p.numel(), ALIGN)
        self.used = sum(s.numel for s in self.slots)          # reference ravel length
        self.numel = _round_up(max(off, ALIGN), pad_multiple)  # padded flat length
        self.p32 = torch.zeros(self.numel, dtype=torch.float32, device=dev)
        self.g32 = torch.zeros(self.numel, dtype=torch.float32, device=dev) if with_grads else None
        self.shadow_dtype = shadow_dtype
        self.w16 = (torch.zeros(self.numel, dtype=shadow_dtype, device=dev)
                    if shadow_dtype is not None else None)
        self._ready_cb = None
        # bumped whenever the bf16 shadow may have changed; keys the cache of
        # transposed conv weights used by the data-gradient kernels
        self.version = 0
        self._wt = None
        self._wt_version = -1
        self._wt_table = None
        self._wt_max = 0
        with torch.no_grad():
            for p, s in zip(self.params, self.slots):
                cl = channels_last and p.dim() == 4
                view = _strided_view(self.p32, s.offset, p, cl)
                view.copy_(p.detach().to(torch.float32))
                p.data = view
                if self.g32 is not None:
                    p.grad = _strided_view(self.g32, s.offset, p, cl)
                p._dmp_arena = True
                p._dmp_arena_ref = weakref.ref(self)
                if self.w16 is not None:
                    p._dmp_w16 = _strided_view(self.w16, s.offset, p, cl)
        self.refresh_shadow()

    # ------------------------------------------------------------------ views
    def param_view(self, i: int) -> torch.Tensor:
        return self.params[i].data

    def flat(self, grads: bool = False) -> torch.Tensor:
        return self.g32 if grads else self.p32

    # ----------------------------------------------------------------- shadow
    def bump(self):
        self.version += 1

    def transposed_conv_shadow(self, p: torch.Tensor):
        """bf16 ``[CI, R, S, CO]`` transpose of conv weight ``p``'s shadow.

        All 4-D weights are transposed together in ONE kernel launch the first
        time this is called after the shadow changed (instead of one launch per
        conv per backward).
        """
        if self.w16 is None or not self.w16.is_cuda:
            return None
        if self._wt is None:
            rows = []
            self._wt_index = {}
            for s, q in zip(self.slots, self.params):
                if len(s.shape) == 4 and s.shape[0] % 64 == 0 and s.shape[1] % 64 == 0:
                    co, ci, r, k = s.shape
                    self._wt_index[id(q)] = s
                    rows.append([s.offset, co, r * k, ci])
                    self._wt_max = max(self._wt_max, s.numel)
            self._wt = torch.empty_like(self.w16)
            self._wt_table = torch.tensor(rows, dtype=torch.int64).reshape(-1, 4).to(self.device)
        s = self._wt_index.get(id(p))
        if s is None:
            return None
        if self._wt_version != self.version:
            from ..ops._ext import native

            native().conv_weight_transpose_batched(self.w16, self._wt, self._wt_table,
                                                   self._wt_max)
            self._wt_version = self.version
        co, ci, r, k = s.shape
        return self._wt[s.offset:s.offset + s.numel].view(ci, r, k, co)

    def padded_rows_shadow(self, p: torch.Tensor, kp: int):
        """bf16 ``[CO, Kp]`` image of conv weight ``p``'s shadow with its rows
        (channels-last ``(r, s, ci)`` order, ``K = R*S*CI``) padded to ``kp``
        columns -- the operand of the im2col GEMM when ``K % 8 != 0`` (LeNet).

        Every such weight lives in one buffer whose pad columns are zeroed once;
        all of them are refreshed by ONE native launch the first time this is
        called after the shadow changed (no per-step fill + copy kernels)."""
        if self.w16 is None or not self.w16.is_cuda:
            return None
        if getattr(self, "_pad", None) is None:
            rows, self._pad_index, off, mx = [], {}, 0, 0
            for s, q in zip(self.slots, self.params):
                if len(s.shape) == 4:
                    co, ci, r, k = s.shape
                    K = ci * r * k
                    Kp = (K + 7) // 8 * 8
                    if K != Kp:
                        self._pad_index[id(q)] = (off, co, Kp)
                        rows.append([s.offset, off, co, K, Kp])
                        off += co * Kp
                        mx = max(mx, co * K)
            self._pad = torch.zeros(max(off, 8), dtype=self.w16.dtype, device=self.device)
            self._pad_table = (torch.tensor(rows, dtype=torch.int64).reshape(-1, 5)
                               .to(self.device))
            self._pad_max = mx
            self._pad_version = -1
        ent = self._pad_index.get(id(p))
        if ent is None or ent[2] != kp:
            return None
        if self._pad_version != self.version:
            from ..ops._ext import native

            native().pad_rows_batched(self.w16, self._pad, self._pad_table, self._pad_max)
            self._pad_version = self.version
        off, co, Kp = ent
        return self._pad[off:off + co * Kp].view(co, Kp)

    def refresh_shadow(self):
        self.bump()
        if self.w16 is None:
            return
        if self.p32.is_cuda:
            from ..ops._ext import native

            native().cast_f32_bf16(self.p32, self.w16)
        else:
            self.w16.copy_(self.p32)

    # ------------------------------------------------------------------ grads
    def zero_grad(self):
        # a new step begins: the shadow may have been rewritten by the update /
        # a pull landing since the last backward
        self.bump()
        if self.g32 is not None:
            if self.g32.is_cuda:
                from ..ops._ext import native

                native().zero_(self.g32)      # native fill kernel (not a graph memset node)
            else:
                self.g32.zero_()

    def ensure_grads_attached(self):
        """Re-attach grad views if user code set ``p.grad = None``."""
        if self.g32 is None:
            return
        for p, s in zip(self.params, self.slots):
            if p.grad is None or p.grad.data_ptr() != self.g32.data_ptr() + 4 * s.offset:
                cl = self.channels_last and p.dim() == 4
                p.grad = _strided_view(self.g32, s.offset, p, cl)

    def set_grad_ready_callback(self, cb):
        """``cb(param_index)`` is called as each parameter's gradient becomes final."""
        self._ready_cb = cb
        for i, p in enumerate(self.params):
            def _ready(_p, _i=i):
                if self._ready_cb is not None:
                    self._ready_cb(_i)
            p._dmp_grad_ready = _ready
            if not hasattr(p, "_dmp_hook_handle"):
                p._dmp_hook_handle = p.register_post_accumulate_grad_hook(
                    lambda t: t._dmp_grad_ready(t) if getattr(t, "_dmp_grad_ready", None) else None)

    # ----------------------------------------------------- ravel compatibility
    def ravel(self, grads: bool = False) -> torch.Tensor:
        """Unpadded concatenation in ``model.parameters()`` order (reference layout)."""
        src = [p.grad if grads else p.data for p in self.params]
        return torch.cat([t.reshape(-1) for t in src])

    def unravel(self, flat: torch.Tensor):
        flat = flat.to(self.device)
        with torch.no_grad():
            if flat.numel() == self.numel:
                self.p32.copy_(flat)
            elif flat.numel() == self.used:
                o = 0
                for p, s in zip(self.params, self.slots):
                    p.data.copy_(flat[o:o + s.numel].view(s.shape))
                    o += s.numel
            else:
                raise ValueError(f"flat vector has {flat.numel()} elements; expected "
                                 f"{self.used} (ravel) or {self.numel} (arena)")
        self.refresh_shadow()

    def state_dict(self):
        return {"p32": self.p32.detach().cpu(), "used": self.used, "numel": self.numel}

    def load_state_dict(self, sd):
        self.unravel(sd["p32"])


def attach_arena(model: torch.nn.Module, **kw) -> FlatArena:
    arena = FlatArena(list(model.parameters()), **kw)
    model._dmp_arena_obj = arena
    return arena


def get_arena(model: torch.nn.Module) -> FlatArena | None:
    return getattr(model, "_dmp_arena_obj", None)
