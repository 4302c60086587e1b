"""Synchronous data parallelism: bucketed all-reduce over the flat grad arena.

New capability (BASELINE.json config #4 "ResNet-50 sync all-reduce DP"); the
reference has no collective at all.  Design:

* gradients already live in ONE flat fp32 buffer (``FlatArena.g32``), so a
  bucket is just a contiguous slice - no gradient copy-in/copy-out;
* buckets are cut in REVERSE parameter order (the order backward produces
  gradients) at ``bucket_mb`` boundaries; each bucket's all-reduce is launched
  from the gradient-ready callback the moment its last gradient lands, so the
  RCCL ring overlaps the rest of backward;
* bucket size MEASURED on the node it runs on (``bucket_mb <= 0``, the default:
  :func:`calibrate_bucket_mb`): on an 8-GPU MI355X node each GPU has 7 xGMI
  links of ~153 GB/s and RCCL splits one all-reduce across channels / links, so
  a bucket must be large enough that each link carries several MB per
  collective while small enough that the last bucket (the tail
  that cannot overlap) stays short.  Where that knee sits depends on the
  topology, world size and RCCL's channel count, so every rank times the
  all-reduce of a few candidate sizes on the real group at start-up, the ranks
  agree on the slowest timing (MAX all-reduce), and the smallest size reaching
  90 % of the best bus bandwidth is the bucket.  ``--bucket-mb X > 0`` pins it;
* the 1/W average is folded into the optimizer's learning rate scale.
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist
from torch.optim.optimizer import Optimizer

from .arena import FlatArena


_CAL_MB = (2.0, 4.0, 8.0, 16.0, 32.0, 64.0)


def calibrate_bucket_mb(group=None, device=None, candidates=_CAL_MB, cap_mb: float | None = None,
                        reps: int = 5, efficiency: float = 0.9):
    """Pick the all-reduce bucket size on the live group -> ``(bucket_mb, table)``.

    ``table`` rows are ``(mb, ms, busbw_GBps)`` with ring bus bandwidth
    ``2 (W-1)/W * bytes / t``; every rank returns the same choice (timings are
    MAX-reduced before deciding).  World 1: nothing to measure, 32 MB."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world <= 1:
        return 32.0, []
    cuda = device is not None and torch.device(device).type == "cuda"
    cands = [c for c in candidates if cap_mb is None or c <= cap_mb] or [min(candidates)]
    buf = torch.zeros(int(max(cands) * 1024 * 1024 / 4), dtype=torch.float32,
                      device=device if cuda else "cpu")
    times = []
    for mb in cands:
        view = buf[: int(mb * 1024 * 1024 / 4)]
        dist.all_reduce(view, group=group)          # warm (RCCL channel setup)
        if cuda:
            torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for _ in range(reps):
            dist.all_reduce(view, group=group)
        if cuda:
            torch.cuda.synchronize(device)
        times.append((time.perf_counter() - t0) / reps)
    t = torch.tensor(times, dtype=torch.float64, device=buf.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)   # one decision on every rank
    times = t.tolist()
    table = []
    for mb, sec in zip(cands, times):
        bw = 2.0 * (world - 1) / world * mb * 1024 * 1024 / max(sec, 1e-9) / 1e9
        table.append((mb, round(sec * 1e3, 4), round(bw, 1)))
    best = max(r[2] for r in table)
    pick = next(r[0] for r in table if r[2] >= efficiency * best)
    return pick, table


class BucketedAllReduce:
    def __init__(self, arena: FlatArena, group=None, bucket_mb: float = 0.0,
                 overlap: bool = True, force_collectives: bool = False):
        """``bucket_mb <= 0``: measured on the group (:func:`calibrate_bucket_mb`,
        capped at half the gradient arena so at least two buckets overlap backward)."""
        self.arena = arena
        self.force = force_collectives
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.overlap = overlap
        self.calibration = []
        if bucket_mb <= 0:
            if self.world > 1:
                half = arena.numel * 4 / (1024 * 1024) / 2
                bucket_mb, self.calibration = calibrate_bucket_mb(
                    group, arena.device, cap_mb=max(half, min(_CAL_MB)))
            else:
                bucket_mb = 32.0
        self.bucket_mb = float(bucket_mb)
        cap = max(int(bucket_mb * 1024 * 1024 / 4), 1)
        # reverse-order buckets of whole parameters: (lo, hi, param indices); the
        # padding after a parameter belongs to it, the arena tail to the last one.
        buckets = []
        hi = arena.numel
        cur, cur_lo = [], hi
        for s in reversed(arena.slots):
            if cur and (hi - s.offset) > cap:
                buckets.append((cur_lo, hi, cur))
                hi, cur = cur_lo, []
            cur.append(s.index)
            cur_lo = s.offset
        if cur:
            buckets.append((cur_lo, hi, cur))
        self.buckets = buckets
        self.owner = {}
        for b, (_, _, idxs) in enumerate(buckets):
            for i in idxs:
                self.owner[i] = b
        self._reset()
        arena.set_grad_ready_callback(self._ready)

    def _reset(self):
        self.remaining = [len(b[2]) for b in self.buckets]
        self.works = [None] * len(self.buckets)
        self.seen = set()

    def reset(self):
        """Forget launched-but-unwaited buckets (after an aborted step / capture)."""
        self._reset()

    def _launch(self, b: int):
        if self.works[b] is not None or (self.world == 1 and not self.force):
            return
        lo, hi, _ = self.buckets[b]
        view = self.arena.g32[lo:hi]
        self.works[b] = dist.all_reduce(view, group=self.group, async_op=True)

    def _ready(self, i: int):
        if not self.overlap or i in self.seen:
            return
        self.seen.add(i)
        b = self.owner[i]
        self.remaining[b] -= 1
        if self.remaining[b] == 0:
            self._launch(b)

    def synchronize(self):
        """Launch any bucket not yet launched, then wait (stream-wait on GPU)."""
        for b in range(len(self.buckets)):
            self._launch(b)
        for w in self.works:
            if w is not None:
                w.wait()
        self._reset()

    @property
    def num_buckets(self) -> int:
        return len(self.buckets)


class FusedSGD(Optimizer):
    """Plain/momentum SGD over a flat arena in one fused HIP kernel.

    Used by sync-DP (with ``grad_scale = 1/world``) and by the reference's
    ``--no-distributed`` baseline (``optim.SGD(lr, momentum=0)``, main.py:43-44).
    """

    def __init__(self, params, arena: FlatArena, lr: float, momentum: float = 0.0,
                 dampening: float = 0.0, nesterov: bool = False, weight_decay: float = 0.0,
                 grad_scale: float = 1.0):
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening,
                                      nesterov=nesterov, weight_decay=weight_decay))
        self.arena = arena
        self.grad_scale = grad_scale
        self.mom = torch.zeros_like(arena.p32) if momentum else None
        self._mom_steps = 0
        self._nat = None
        if arena.device.type == "cuda":
            from ..ops._ext import native

            self._nat = native()

    def zero_grad(self, set_to_none: bool = False):
        self.arena.ensure_grads_attached()
        self.arena.zero_grad()

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self.local_step()
        return loss

    def comm_step(self):
        pass

    @torch.no_grad()
    def local_step(self):
        g = self.param_groups[0]
        a = self.arena
        lr = g["lr"]
        a.bump()
        if self.grad_scale != 1.0:
            # fold the 1/W average into lr (and rescale weight decay so wd*p is not scaled)
            lr_eff = lr * self.grad_scale
            wd_eff = g["weight_decay"] / self.grad_scale
        else:
            lr_eff, wd_eff = lr, g["weight_decay"]
        if self.mom is not None and self.grad_scale != 1.0:
            # momentum must see the averaged gradient: scale grads explicitly
            a.g32.mul_(self.grad_scale)
            lr_eff, wd_eff = lr, g["weight_decay"]
        # first update: momentum buffer = gradient, as torch.optim.SGD (no dampening)
        damp = g["dampening"] if self._mom_steps > 0 else 0.0
        self._mom_steps += 1
        if self._nat is not None:
            self._nat.asgd_fused_step(a.g32, a.p32, None, self.mom, a.w16, lr_eff, wd_eff,
                                      g["momentum"], damp, g["nesterov"])
        else:
            d = a.g32
            if wd_eff:
                d = d + wd_eff * a.p32
            if self.mom is not None:
                self.mom.mul_(g["momentum"]).add_(d, alpha=1 - damp)
                d = d + g["momentum"] * self.mom if g["nesterov"] else self.mom
            a.p32.add_(d, alpha=-lr_eff)
            if a.w16 is not None:
                a.w16.copy_(a.p32)
