"""Non-lock-step sharded parameter server (``--ps sharded_async``).

:class:`~.clients.ShardedPSClient` moves pushes and pulls with collectives
(reduce-scatter / all-gather): every rank must join every push, so one late
rank stalls the node at its next due pull -- bounded-staleness periodic
averaging rather than Downpour asynchrony.  Here the master is still split
into one shard per rank, but each shard is a small parameter server of its own
(DistBelief's sharded PS, /root/reference/asgd/optim/Asynchronous.py:48-70
generalised from one PS rank to N co-located shards):

* a :class:`ShardServer` thread per rank owns ``master[lo_r:hi_r]`` and serves
  ``GradientUpdate`` (``shard += scale * delta``, applied the moment it
  arrives, whoever sent it) and ``ParameterRequest`` (reply with a snapshot
  and the shard version) to ANY rank's worker, using the typed header/payload
  protocol of :mod:`.messaging` (any-source header receive, per-sender payload);
* a worker's push sends each shard owner its slice of the accumulated delta
  (point-to-point, fire-and-forget, tracked) and applies its own slice
  in-process; a pull requests every shard and lands, ``staleness`` steps
  later, whatever versions the owners had when they answered.

Nothing is a collective after the initial broadcast: a slow or paused rank
delays only the replies of its own shard (its server thread keeps serving
while its worker computes) and never blocks another rank's push.  Traffic is
gloo point-to-point on two dedicated groups (requests, replies); on GPUs the
payloads are host-staged -- the option trades bandwidth for independence.
"""
from __future__ import annotations

import logging
import threading
from collections import Counter

import torch
import torch.distributed as dist

from . import messaging as M
from .clients import PSClient, _Pending

_LOG = logging.getLogger(__name__)


class ShardServer:
    """One rank's shard of the master, served to every rank from a thread."""

    def __init__(self, rank: int, world: int, init_shard: torch.Tensor, req_group, rep_group,
                 scale: float = 1.0):
        self.rank, self.world = rank, world
        self.master = init_shard.detach().to(torch.float32).clone()
        self.req, self.rep = req_group, rep_group
        self.scale = scale
        self.lock = threading.Lock()
        self.version = 0
        self.counts: Counter = Counter()
        self.staleness: list[int] = []
        self.tracker = M.SendTracker()
        self.error: BaseException | None = None
        self.thread = threading.Thread(target=self._run, daemon=True, name=f"shard-ps-{rank}")

    def start(self):
        self.thread.start()
        return self

    # called from the server thread (remote pushes) and the local worker
    def apply(self, delta: torch.Tensor, base_version: int | None = None):
        with self.lock:
            self.master.add_(delta.to(torch.float32), alpha=self.scale)
            if base_version is not None:
                self.staleness.append(self.version - base_version)
            self.version += 1

    def snapshot(self) -> tuple[torch.Tensor, int]:
        with self.lock:
            return self.master.clone(), self.version

    def _run(self):
        remaining = set(range(self.world)) - {self.rank}
        n = self.master.numel()
        try:
            while remaining:
                code, sender, _step, version, nelem, dtype = M.recv_header(None, self.req)
                self.counts[code.name] += 1
                if code == M.MessageCode.GradientUpdate:
                    if nelem != n:
                        raise RuntimeError(f"shard {self.rank}: rank {sender} pushed {nelem} "
                                           f"elements, the shard has {n}")
                    buf = torch.empty(nelem, dtype=dtype)
                    dist.recv(buf, src=sender, group=self.req, tag=M.TAG_PAYLOAD)
                    self.apply(buf, version)
                elif code == M.MessageCode.ParameterRequest:
                    snap, v = self.snapshot()
                    out = torch.cat([snap, torch.tensor([float(v)])])
                    self.tracker.add(dist.isend(out, sender, group=self.rep, tag=M.TAG_REPLY), out)
                elif code == M.MessageCode.Shutdown:
                    remaining.discard(sender)
        except BaseException as e:   # surfaced by join()
            self.error = e

    def join(self):
        self.thread.join()
        self.tracker.drain()
        if self.error is not None:
            raise RuntimeError(f"shard server {self.rank} failed: {self.error!r}")

    def stats(self) -> dict:
        st = self.staleness
        return {"shard_version": self.version, "shard_counts": dict(self.counts),
                "shard_staleness_mean": (sum(st) / len(st)) if st else 0.0,
                "shard_staleness_max": max(st) if st else 0}


class _ShardedPull:
    """Work over the per-shard replies of one pull: ``wait()`` assembles them
    (plus the local shard's snapshot, already in place) into the flat buffer."""

    def __init__(self, buf, parts):
        self.buf, self.parts, self.done = buf, parts, False
        self.versions: list[int] = []

    def wait(self):
        if not self.done:
            for lo, hi, rbuf, work in self.parts:
                work.wait()
                self.buf[lo:hi].copy_(rbuf[: hi - lo])
                self.versions.append(int(rbuf[hi - lo].item()))
            self.done = True
        return True


class AsyncShardedPSClient(PSClient):
    """Worker side of the non-lock-step sharded PS (one :class:`ShardServer` per rank)."""

    def __init__(self, group=None, delta_scale: str | float = "sum", **kw):
        """``delta_scale``: ``"sum"`` adds every worker's delta as a Downpour PS
        does; ``"mean"`` scales each delta by 1/world; a float is used as is."""
        super().__init__(**kw)
        self.group = group
        self.delta_scale = delta_scale
        self.shard_versions: list[int] = []

    def init(self):
        self.world = dist.get_world_size(self.group)
        self.rank = dist.get_rank(self.group)
        n = self.arena.numel
        if n % self.world:
            raise ValueError(f"arena length {n} not divisible by world size {self.world}")
        self.shard_n = n // self.world
        scale = {"sum": 1.0, "mean": 1.0 / self.world}.get(self.delta_scale)
        scale = float(self.delta_scale) if scale is None else scale
        # identical start everywhere, then no collective ever again
        dist.broadcast(self.arena.p32, 0, group=self.group)
        self.arena.refresh_shadow()
        # every rank creates both groups in the same order (torch new_group rule)
        self.req = dist.new_group(list(range(self.world)), backend="gloo")
        self.rep = dist.new_group(list(range(self.world)), backend="gloo")
        # host barriers (resume) on a group of their own: the shard servers keep an
        # any-source receive posted on `req` at all times
        self.ctl = dist.new_group(list(range(self.world)), backend="gloo")
        lo = self.rank * self.shard_n
        init = self.arena.p32.detach()[lo: lo + self.shard_n].cpu()
        self.server = ShardServer(self.rank, self.world, init, self.req, self.rep, scale).start()

    def _bounds(self, o: int):
        return o * self.shard_n, (o + 1) * self.shard_n

    def push(self, step: int):
        buf = self._handoff()
        self._resolve_versions()
        # a private host copy: gloo reads an unbound send buffer only when the
        # owner posts its receive, and the hand-off slot is refilled two pushes on
        host = buf.detach().to("cpu", copy=True)
        for o in range(self.world):
            lo, hi = self._bounds(o)
            if o == self.rank:
                self.server.apply(host[lo:hi], self.version)
            else:
                M.send_message(M.MessageCode.GradientUpdate, host[lo:hi], o, step=step,
                               version=self.version, group=self.req)
        self.pushes += 1
        self.bytes_sent += host.numel() * host.element_size() * (self.world - 1) // self.world

    def request_pull(self, step: int):
        n = self.arena.numel
        buf = torch.empty(n, dtype=torch.float32)
        parts = []
        for o in range(self.world):
            lo, hi = self._bounds(o)
            if o == self.rank:
                snap, _ = self.server.snapshot()
                buf[lo:hi].copy_(snap)
                continue
            M.send_message(M.MessageCode.ParameterRequest, None, o, step=step, group=self.req)
            rbuf = torch.empty(hi - lo + 1, dtype=torch.float32)
            work = M.OnceWork(dist.irecv(rbuf, o, group=self.rep, tag=M.TAG_REPLY))
            parts.append((lo, hi, rbuf, work))
        self.pending.append(_Pending(step, buf, work=_ShardedPull(buf, parts)))
        self.bytes_recv += n * 4 * (self.world - 1) // self.world

    def _land(self, pend):
        pend.work.wait()
        self.shard_versions = pend.work.versions
        if pend.work.versions:
            self.version = max(self.version, min(pend.work.versions))
        pend.work = None
        if self.cuda:
            pend.buf = pend.buf.to(self.device, non_blocking=False)
        super()._land(pend)

    def finish(self):
        super().finish()                       # lands every requested pull
        for o in range(self.world):
            if o != self.rank:
                M.send_message(M.MessageCode.Shutdown, None, o, group=self.req)
        M.SENDS.drain()
        self.server.join()                     # returns once every rank has shut down

    def stats(self) -> dict:
        st = super().stats()
        st.update(self.server.stats())
        return st

    @property
    def master(self) -> torch.Tensor:
        return self.server.master

    def state_dict(self) -> dict:
        snap, v = self.server.snapshot()
        return {"kind": "sharded_async", "rank": self.rank, "world": self.world,
                "master": snap, "shard_version": v}

    def load_state_dict(self, sd: dict):
        if sd.get("kind") != "sharded_async":
            return
        if sd["world"] != self.world or sd["rank"] != self.rank:
            raise ValueError(f"sharded PS checkpoint is for rank {sd['rank']}/{sd['world']}, "
                             f"this is rank {self.rank}/{self.world}")
        with self.server.lock:
            self.server.master.copy_(sd["master"])
            self.server.version = int(sd.get("shard_version", 0))
        # every shard restored before anyone asks for it: without this barrier a
        # fast rank's forced pull could be answered with a peer's pre-restore shard
        dist.barrier(group=self.ctl)
        # re-sync the live parameters from every restored shard
        self.request_pull(0)
        self.land_due(0, force=True)
        self.arena.refresh_shadow()
