"""``ravel_model_params`` / ``unravel_model_params`` (reference C10).

Contract reconstructed from the call sites in
/root/reference/asgd/optim/Asynchronous.py:18,27,34,54 (module missing
upstream):

* ``ravel_model_params(model, grads=False)`` -> 1-D fp32 tensor concatenating
  every ``p.data`` (or ``p.grad``) in ``model.parameters()`` order; buffers
  (BN running stats) are not included.
* ``unravel_model_params(model, flat)`` copies consecutive slices back in place.

When the model has a :class:`FlatArena` attached, ``zero_copy=True`` returns the
arena's padded flat buffer itself (no concatenation), and ``unravel`` accepts
either length.
"""
from __future__ import annotations

import torch

from ..parallel.arena import get_arena


def ravel_model_params(model: torch.nn.Module, grads: bool = False, zero_copy: bool = False):
    arena = get_arena(model)
    if arena is not None:
        if zero_copy:
            return arena.flat(grads)
        return arena.ravel(grads)
    parts = []
    for p in model.parameters():
        t = p.grad if grads else p.data
        if t is None:
            t = torch.zeros_like(p.data)
        parts.append(t.reshape(-1).to(torch.float32))
    return torch.cat(parts)


def unravel_model_params(model: torch.nn.Module, flat: torch.Tensor):
    arena = get_arena(model)
    if arena is not None:
        arena.unravel(flat)
        return
    o = 0
    with torch.no_grad():
        for p in model.parameters():
            n = p.numel()
            p.data.copy_(flat[o:o + n].view_as(p.data).to(p.dtype))
            o += n
    if o != flat.numel():
        raise ValueError(f"flat vector has {flat.numel()} elements, model has {o}")


def num_params(model: torch.nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())
