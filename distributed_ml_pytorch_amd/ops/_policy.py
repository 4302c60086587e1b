"""Where a stock (ATen / MIOpen / hipBLASLt) kernel may run on a GPU tensor.

The framework's GPU path is its own gfx950 kernels (``csrc/*.hip``).  Every op
of ``ops`` that would hand a CUDA tensor to a stock kernel -- an fp32 input, a
geometry no native kernel covers (head dim != 64 attention, a conv shape
outside the tiles), ... -- calls :func:`stock_gpu` first, and by default that
RAISES: a model that leaves native coverage fails loudly instead of training on
MIOpen / hipBLASLt without anyone noticing (VERDICT r5 weakness #7, the
loader's contract in ``ops/_ext.py``).

The one exception is the explicit stock ORACLE mode -- ``--deterministic``
(``runtime/determinism.py``: fp32 on PyTorch's deterministic kernels, the
reference trajectory the native path is compared against) and the fp32
numerics oracles of the test suite -- entered with :func:`allow_stock` /
:func:`stock_allowed`.  In that mode every distinct (op, reason) that goes to
a stock kernel is logged once, so a run records which layers it sent there.
CPU tensors are never affected (gloo plumbing runs, CPU tests).
"""
from __future__ import annotations

import contextlib
import logging
import threading

import torch

_LOG = logging.getLogger(__name__)
# overrides of stock_allowed() blocks, innermost last.  Process-wide, not
# thread-local: the autograd engine runs a CUDA backward on its own device
# thread, and a block's setting must hold for the backward it launches too.
_overrides: list = []
_global_allow = False
_seen: set = set()
_lock = threading.Lock()


class NativeCoverageError(RuntimeError):
    """A GPU tensor reached an op outside native kernel coverage."""


def allow_stock(on: bool = True, reason: str = "stock oracle mode"):
    """Process-wide switch (``--deterministic``)."""
    global _global_allow
    _global_allow = bool(on)
    if on:
        _LOG.warning("stock GPU kernels allowed: %s (layers sent there are logged once each)",
                     reason)


@contextlib.contextmanager
def stock_allowed(on: bool = True):
    """Override for a block, including the backward passes it runs (tests: fp32
    oracles on the GPU; the strict all-native test sets ``on=False``)."""
    with _lock:
        _overrides.append(bool(on))
    try:
        yield
    finally:
        with _lock:
            _overrides.pop()


def is_allowed() -> bool:
    with _lock:
        return _overrides[-1] if _overrides else _global_allow


def stock_log() -> list:
    """(op, reason) pairs sent to stock kernels so far (oracle mode only)."""
    with _lock:
        return sorted(_seen)


def stock_gpu(op: str, *tensors, reason: str = ""):
    """Gate a stock kernel call: no-op unless one of ``tensors`` is on the GPU;
    then raise outside the oracle mode, log the (op, reason) once inside it."""
    t = next((x for x in tensors if torch.is_tensor(x) and x.is_cuda), None)
    if t is None:
        return
    why = reason or f"dtype {t.dtype}, shape {tuple(t.shape)}"
    if not is_allowed():
        raise NativeCoverageError(
            f"{op}: no native gfx950 kernel covers this GPU input ({why}); refusing to run a "
            "stock ATen / MIOpen / hipBLASLt kernel silently.  The native path is bf16 "
            "compute; stock fp32 kernels run only in the explicit oracle mode "
            "(--deterministic, or ops._policy.stock_allowed())")
    key = (op, why)
    with _lock:
        new = key not in _seen
        _seen.add(key)
    if new:
        _LOG.warning("stock GPU kernel: %s (%s)", op, why)
