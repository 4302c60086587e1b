"""Opt-in bitwise-reproducible debugging mode (``--deterministic``).

Why it exists: the native bf16 path is fast partly BECAUSE its split
reductions are order-free -- the conv / GEMM weight gradients split the pixel
(or token) reduction over hundreds of blocks and add their fp32 partials with
memory-side atomics, and the BatchNorm statistics arrive as per-block sums
atomically added into 64 slots (csrc/bn_slots.h).  fp32 addition is not
associative, so two runs of the same step differ in the last bits, and after a
few hundred steps ASGD and sync-DP trajectories diverge by more than the
effect one is usually hunting (tests/test_train_gpu.py tolerates a loss delta
of 5e-2 between graph and eager runs for this reason).

What the mode does (:func:`enable_determinism`):

* compute in fp32 on PyTorch's own kernels -- the framework's fp32 oracle
  path (``--dtype fp32``: ops/functional.py routes every fp32 GPU op to ATen /
  MIOpen / hipBLASLt) -- with ``torch.use_deterministic_algorithms(True)``
  (errors, not warnings: an op without a deterministic implementation stops
  the run instead of silently breaking the guarantee), MIOpen's deterministic
  algorithm selection (``cudnn.deterministic``, no benchmark autotuning) and
  PyTorch's fixed BLAS workspace (``CUBLAS_WORKSPACE_CONFIG``, which PyTorch
  reads for its hipBLAS(Lt) handles on ROCm too; set before any handle exists),
  so no kernel reduces through atomics;
* keep everything else of the framework unchanged: the flat fp32 arena, the
  fused elementwise optimizer kernels (one thread per element: deterministic),
  the PS machinery and its push/pull cadence, the hipGraph capture.

What stays non-deterministic by design: the ORDER in which an asynchronous
central PS applies pushes from several workers (that is the algorithm); with a
local PS, sync DP (RCCL ring all-reduce over a fixed world is reproducible) or
one worker, runs are bitwise identical.  The cost is speed -- fp32 on stock
kernels, roughly the stock-PyTorch column of profiles/stock_vs_ours_r2.txt --
which is the point: this is the reference trajectory the fast path is
compared against, not a production setting.
"""
from __future__ import annotations

import dataclasses
import logging
import os

import torch

_LOG = logging.getLogger(__name__)


def enable_determinism(cfg):
    """Switch the process to deterministic kernels; return ``cfg`` with fp32 compute."""
    os.environ.setdefault("CUBLAS_WORKSPACE_CONFIG", ":4096:8")
    torch.use_deterministic_algorithms(True, warn_only=False)
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
    # the one mode in which GPU ops may run on stock kernels: each (op, reason)
    # sent there is logged once (ops/_policy.py)
    from ..ops._policy import allow_stock

    allow_stock(True, "--deterministic (fp32 on PyTorch's deterministic kernels)")
    if cfg.dtype != "fp32":
        _LOG.info("deterministic mode: compute dtype %s -> fp32 (PyTorch deterministic kernels)",
                  cfg.dtype)
        cfg = dataclasses.replace(cfg, dtype="fp32")
    return cfg


def is_enabled() -> bool:
    return torch.are_deterministic_algorithms_enabled()
