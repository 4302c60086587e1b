"""Downpour / asynchronous SGD optimizer (reference C1 + C8).

Worker side of DistBelief Downpour SGD, re-implemented from the behaviour of
/root/reference/asgd/optim/Asynchronous.py:20-71:

* every ``n_pull`` steps request the PS parameters (:48-49),
* accumulate ``-lr * grad`` into a push accumulator (:54-55),
* every ``n_push`` steps send the accumulator to the PS and zero it (:58-60),
* always apply the local SGD step ``p -= lr * grad`` (:63-68).

What is different by design:

* one fused HIP kernel over the flat arena does accumulate + local step +
  bf16 shadow refresh (no per-step ravel ``torch.cat``, no per-tensor loop);
* the accumulator lives on the parameters' device (D4);
* a pulled snapshot is landed at a step boundary by the optimizer itself,
  never written into live parameters by a listener thread (D13), and at most
  ``staleness`` steps after it was requested (bounded staleness);
* ``super().__init__`` is called correctly (D2) and ``DownpourSGD`` is exported
  (D1).
"""
from __future__ import annotations

import torch
import torch.distributed as dist
from torch.optim.optimizer import Optimizer, required

from .arena import attach_arena, get_arena
from .clients import GlooPSClient, LocalPSClient, PSClient


def default_client(**kw) -> PSClient:
    """The reference's implicit choice: rank 0 is the PS over gloo, else local."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return GlooPSClient(ps_rank=0, **kw)
    return LocalPSClient(**kw)


class Asynchronous(Optimizer):
    def __init__(self, params, lr=required, n_push=required, n_pull=required, model=required, *,
                 client: PSClient | None = None, staleness: int = 1, momentum: float = 0.0,
                 dampening: float = 0.0, nesterov: bool = False, weight_decay: float = 0.0,
                 pull_mode: str = "overwrite", wire_dtype: torch.dtype = torch.float32,
                 shadow_dtype: torch.dtype | None | str = "auto"):
        if lr is required or n_push is required or n_pull is required or model is required:
            raise TypeError("Asynchronous needs lr, n_push, n_pull and model")
        if lr < 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if int(n_push) < 1 or int(n_pull) < 1:
            raise ValueError("n_push and n_pull must be >= 1")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, nesterov=nesterov,
                        weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.model = model
        self.n_push = int(n_push)
        self.n_pull = int(n_pull)
        arena = get_arena(model)
        if arena is None:
            dev = next(model.parameters()).device
            if shadow_dtype == "auto":
                shadow_dtype = torch.bfloat16 if dev.type == "cuda" else None
            arena = attach_arena(model, shadow_dtype=shadow_dtype)
        self.arena = arena
        mine = {id(p) for g in self.param_groups for p in g["params"]}
        if mine != {id(p) for p in arena.params}:
            raise ValueError("Asynchronous must be given exactly model.parameters() "
                             "(the push/pull vector is the whole model, as in the reference)")
        dev = arena.device
        self.acc = torch.zeros(arena.numel, dtype=torch.float32, device=dev)
        self._mom_steps = 0
        self.mom = torch.zeros_like(self.acc) if momentum else None
        self.idx = 0
        self.timer = _NO_TIMER      # a utils.metrics.StepTimer when the trainer wires one
        self.client = client if client is not None else default_client(
            staleness=staleness, pull_mode=pull_mode, wire_dtype=wire_dtype)
        self.client.attach(self)
        self.client.init()
        self._nat = None
        if dev.type == "cuda":
            from ..ops._ext import native

            self._nat = native()

    # reference-visible attributes -----------------------------------------
    @property
    def accumulated_gradients(self) -> torch.Tensor:
        return self.acc

    def zero_grad(self, set_to_none: bool = False):
        """Zero the flat grad arena (views stay attached; ``set_to_none`` ignored).
        Opens the compute half of a step (closed by ``local_step``)."""
        self.client.in_compute = True
        self.arena.ensure_grads_attached()
        self.arena.zero_grad()

    def _local_update(self, lr: float):
        g = self.param_groups[0]
        a = self.arena
        # torch.optim.SGD seeds the momentum buffer with the first gradient
        # (no dampening); the buffer starts at zero, so dampening 0 on the
        # first update gives exactly that
        damp = g["dampening"] if self._mom_steps > 0 else 0.0
        self._mom_steps += 1
        if self._nat is not None:
            self._nat.asgd_fused_step(a.g32, a.p32, self.acc, self.mom, a.w16, lr,
                                      g["weight_decay"], g["momentum"], damp, g["nesterov"])
            return
        with torch.no_grad():
            d = a.g32
            if g["weight_decay"]:
                d = d + g["weight_decay"] * a.p32
            if self.mom is not None:
                self.mom.mul_(g["momentum"]).add_(d, alpha=1 - damp)
                d = d + g["momentum"] * self.mom if g["nesterov"] else self.mom
            self.acc.add_(d, alpha=-lr)
            a.p32.add_(d, alpha=-lr)
            if a.w16 is not None:
                a.w16.copy_(a.p32)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self.local_step()
        self.comm_step()
        return loss

    @torch.no_grad()
    def local_step(self):
        """Device-only half of a step (graph-capturable): fused accumulate + SGD."""
        self._local_update(self.param_groups[0]["lr"])
        self.arena.bump()
        self.client.in_compute = False

    @torch.no_grad()
    def comm_step(self):
        """Host-scheduled half: push / pull / land on the reference cadence."""
        t = self.timer
        if self.idx % self.n_push == 0:
            with t.time("push"):
                self.client.push(self.idx)
        if self.idx % self.n_pull == 0:
            with t.time("pull_issue"):
                self.client.request_pull(self.idx)
        with t.time("land"):
            self.client.land_due(self.idx)
        self.idx += 1

    def finish(self):
        """Land outstanding pulls, flush sends, tell the PS we are done."""
        self.client.finish()

    def stats(self) -> dict:
        return {"steps": self.idx, **self.client.stats()}


class _NoTimer:
    class _Ctx:
        def __enter__(self):
            return self

        def __exit__(self, *a):
            return False

    _ctx = _Ctx()

    def time(self, name):
        return self._ctx


_NO_TIMER = _NoTimer()


# The reference's package exports this name (asgd/optim/__init__.py:1) while its
# class body is called Asynchronous (Asynchronous.py:40): both names, one class.
DownpourSGD = Asynchronous
