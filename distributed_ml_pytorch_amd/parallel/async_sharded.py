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
  and the shard version) to ANY rank's worker;
* a worker's push sends each shard owner its slice of the accumulated delta
  and applies its own slice in-process; a pull requests every shard and lands,
  ``staleness`` steps later, whatever versions the owners had when they
  answered.

Nothing is a collective after start-up: a slow or paused rank delays only the
replies of its own shard (its server thread keeps serving while its worker
computes) and never blocks another rank's push.

Transport (RCCL has no any-source receive and no tags):

* control -- typed headers (:mod:`.messaging`) on one gloo group, received
  any-source by each shard server;
* payloads -- point-to-point on dedicated 2-rank groups, ONE PER DIRECTION AND
  KIND: ``push[s -> o]`` (worker s's delta slice to shard server o) and
  ``reply[o -> s]`` (server o's snapshot to worker s).  Each group then carries
  sends of one thread on one side and receives of one thread on the other, in
  the same order on both (a header precedes its payload), so no two transfers
  can be matched out of order and no send waits on a receive queued behind it
  on the same communicator.  On GPUs these are RCCL communicators (xGMI): the
  master shards are device-resident, pushes are applied with the native
  ``ps_apply`` kernel on the server's own HIP stream as the receive completes
  (stream-ordered, no host sync), replies are snapshots taken on that stream,
  and pulled shards land in device staging buffers through ``pull_land`` at a
  step boundary -- no host copy anywhere on the payload path, and the server
  thread never blocks on the device (it only blocks, GIL released, in the gloo
  header receive).  On CPU the same groups are gloo groups (the tests).
"""
from __future__ import annotations

import logging
import threading
from collections import Counter, deque

import torch
import torch.distributed as dist

from . import messaging as M
from .clients import PSClient, _EventWork, _Pending
from .links import AppliedCount, PairGroupTransport, PairLinks, wait_on, warm_stream

_LOG = logging.getLogger(__name__)


def make_p2p_groups(world: int, backend: str):
    """``push[(s, o)]`` and ``reply[(o, s)]`` 2-rank groups for every ordered pair
    (every rank must call this, in the same order: torch ``new_group`` rule)."""
    push, reply = {}, {}
    for s in range(world):
        for o in range(world):
            if s == o:
                continue
            push[(s, o)] = dist.new_group(sorted((s, o)), backend=backend)
            reply[(s, o)] = dist.new_group(sorted((s, o)), backend=backend)
    return push, reply


def warm_up_p2p(rank: int, groups: dict, device):
    """One 1-element exchange on every group, in one global order: RCCL
    communicators are created lazily by their first operation and creation is
    collective over the pair, so doing it here (from the main thread, all ranks
    in the same order) keeps it out of the server threads' hot path."""
    for (s, o), g in sorted(groups.items()):
        if rank == s:
            dist.send(torch.ones(1, device=device), o, group=g)
        elif rank == o:
            t = torch.zeros(1, device=device)
            dist.recv(t, s, group=g)


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class ShardServer:
    """One rank's shard of the master, served to every rank from a thread.

    ``push_groups[(sender, rank)]`` / ``reply_groups[(rank, dst)]``: the payload
    groups this server receives pushes on / sends replies on."""

    def __init__(self, rank: int, world: int, init_shard: torch.Tensor, req_group,
                 push_groups: dict, reply_groups: dict, scale: float = 1.0, transport=None):
        self.rank, self.world = rank, world
        self.device = init_shard.device
        self.cuda = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(self.device) if self.cuda else None
        if self.cuda:
            from ..ops._ext import native

            self.nat = native()
            # the shard is a copy of the arena made in the order of the compute stream
            self.stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.stream):
                self.master = init_shard.detach().to(torch.float32).clone()
        else:
            self.master = init_shard.detach().to(torch.float32).clone()
        # link-concurrent payloads (:mod:`.links`): one stream + buffer ring per
        # (peer, direction), so pushes from different ranks land concurrently and
        # (GPU) each is applied on its own link stream as soon as it has landed
        # (fp32 atomics).  The same code path runs on CPU (gloo groups, host
        # waits, applies in arrival order) -- the multi-process tests exercise it.
        peers = [r for r in range(world) if r != rank]
        self.rx = PairLinks(self.device, transport or PairGroupTransport(
            {s: g for (s, _o), g in push_groups.items()}), peers=peers)
        self.tx = PairLinks(self.device, transport or PairGroupTransport(
            {d: g for (_o, d), g in reply_groups.items()}), peers=peers)
        self.req = req_group
        self.push_g = push_groups
        self.reply_g = reply_groups
        self.scale = scale
        self.lock = threading.Lock()
        self.version = 0           # applies ENQUEUED (host): staleness of incoming pushes
        # applies wholly landed (device count on GPU): what a reply is stamped with
        self.applied = AppliedCount(self.device, self.nat if self.cuda else None)
        self.counts: Counter = Counter()
        self.staleness: list[int] = []
        self.error: BaseException | None = None
        self.n = self.master.numel()
        for p in peers:                  # payload rings up front (see PairLinks.reserve)
            for dt in (torch.float32, torch.bfloat16):
                self.rx.reserve(p, self.n, dt)
            self.tx.reserve(p, self.n + 1, torch.float32, send=True)
        if self.cuda and peers:
            # load the apply kernels before any transfer: a kernel's first launch
            # loads its code object, and that waited for the transfers in flight
            # (ParameterServer._warm_kernels); a zero delta changes nothing
            with torch.cuda.stream(self.stream):
                for dt in (torch.float32, torch.bfloat16):
                    self.nat.ps_apply(self.master, torch.zeros(self.n, dtype=dt,
                                                               device=self.device),
                                      None, self.scale, True)
                self.nat.ps_count(self.applied.dev, 0)
                self.nat.ps_stamp(self.applied.dev, torch.empty(1, device=self.device))
            self.stream.synchronize()
        self.thread = threading.Thread(target=self._run, daemon=True, name=f"shard-ps-{rank}")

    def start(self):
        self.thread.start()
        return self

    def _ctx(self):
        return torch.cuda.stream(self.stream) if self.cuda else _Null()

    # --------------------------------------------------------------- apply
    def _apply_locked(self, delta: torch.Tensor, base_version: int | None):
        if self.cuda:
            # fp32 atomics: the local apply (self.stream) and every peer's apply
            # (its own link stream, _recv_push) may run at the same time
            self.nat.ps_apply(self.master, delta, None, self.scale, True)
        else:
            self.master.add_(delta.to(torch.float32), alpha=self.scale)
        self.applied.bump()        # GPU: on the applying stream, counted once landed
        if base_version is not None:
            self.staleness.append(self.version - base_version)
        self.version += 1

    def apply(self, delta: torch.Tensor, base_version: int | None = None):
        """Apply a delta from the calling thread (the co-located worker's own
        slice): on GPU ordered after the caller's current stream, run on the PS
        stream.  Returns the event marking the apply done (GPU; ``None`` on CPU):
        ``delta`` may be overwritten only after it -- ``record_stream`` guards
        the allocation, not a reuse of the same buffer."""
        with self.lock:
            if self.cuda:
                self.stream.wait_stream(torch.cuda.current_stream(self.device))
                with self._ctx():
                    self._apply_locked(delta, base_version)
                    done = torch.cuda.Event()
                    done.record()
                delta.record_stream(self.stream)
                return done
            self._apply_locked(delta, base_version)
            return None

    def snapshot(self, out: torch.Tensor | None = None):
        """``(copy of the shard, version, event)``: on GPU the copy is taken on the
        PS stream after every LOCAL apply enqueued so far (peers' applies land on
        their link streams whenever their payloads arrive); ``event`` marks it done.
        ``version`` counts the applies the copy wholly contains: a host int on CPU,
        on GPU a 1-element device tensor stamped on the PS stream before the copy
        (:class:`.links.AppliedCount`)."""
        with self.lock:
            if not self.cuda:
                snap = self.master.clone() if out is None else out.copy_(self.master)
                return snap, self.applied.host, None
            with self._ctx():
                v = torch.empty(1, dtype=torch.float32, device=self.device)
                self.applied.stamp(v)
                snap = self.master.clone() if out is None else out.copy_(self.master)
                ev = torch.cuda.Event()
                ev.record()
            return snap, v, ev

    # ---------------------------------------------------------------- serve
    def _recv_push(self, sender: int, nelem: int, dtype, version: int):
        if nelem != self.n:
            raise RuntimeError(f"shard {self.rank}: rank {sender} pushed {nelem} elements, "
                               f"the shard has {self.n}")
        # posted on the sender's own link stream, behind nothing but the apply
        # that last read its ring slot; no lock: only the apply needs one
        slot, ready = self.rx.recv(sender, nelem, dtype)
        if self.cuda:
            # completion-ordered: applied on the SENDER's link stream right behind
            # its own receive, so a slow peer's payload still in flight delays no
            # other peer's apply (the receive's ``ready`` is on that stream)
            s = self.rx.stream(sender)
            with self.lock, torch.cuda.stream(s):
                self._apply_locked(slot.buf, version)
                self.rx.release(slot, s)
            return
        with self.lock, self._ctx():
            wait_on(self.stream, ready)
            self._apply_locked(slot.buf, version)
            self.rx.release(slot, self.stream)

    def _reply(self, dst: int):
        n = self.n
        with self.lock:
            def fill(buf):
                self.applied.stamp(buf[n:])    # before the copy: wholly-landed applies
                buf[:n].copy_(self.master)

            # snapshot on dst's own reply-link stream, after dst's own applies
            # (its push-link stream: read-your-writes) and the local worker's
            # (self.stream), never behind another peer's payload in flight; the
            # ring slot is reused only after its previous send completed
            if self.cuda:
                s = self.tx.stream(dst)
                for src in (self.rx.stream(dst), self.stream):
                    ev = torch.cuda.Event()
                    ev.record(src)
                    s.wait_event(ev)
                self.tx.send(dst, n + 1, torch.float32, fill, s)
            else:
                self.tx.send(dst, n + 1, torch.float32, fill, self.stream)

    def _run(self):
        remaining = set(range(self.world)) - {self.rank}
        try:
            while remaining:
                code, sender, _step, version, nelem, dtype = M.recv_header(None, self.req)
                self.counts[code.name] += 1
                if code == M.MessageCode.GradientUpdate:
                    self._recv_push(sender, nelem, dtype, version)
                elif code == M.MessageCode.ParameterRequest:
                    self._reply(sender)
                elif code == M.MessageCode.Shutdown:
                    remaining.discard(sender)
        except BaseException as e:   # surfaced by join()
            self.error = e

    def join(self):
        self.thread.join()
        self.rx.synchronize()
        self.tx.synchronize()
        if self.cuda:
            self.stream.synchronize()
        if self.error is not None:
            raise RuntimeError(f"shard server {self.rank} failed: {self.error!r}")

    def stats(self) -> dict:
        st = self.staleness
        return {"shard_version": self.version, "shard_applied": self.applied.value(),
                "shard_counts": dict(self.counts),
                "shard_links": dict(self.rx.counts, sends=self.tx.counts["send"],
                                    send_reused=self.tx.counts["reused"]),
                "shard_staleness_mean": (sum(st) / len(st)) if st else 0.0,
                "shard_staleness_max": max(st) if st else 0}


class _ShardedPull:
    """The per-shard replies of one pull (plus the local shard's snapshot)."""

    def __init__(self, parts, own, own_version: int = 0):
        self.parts = parts         # [(lo, hi, rbuf [hi - lo + 1], work)]
        self.own = own             # (lo, hi, buf, event)
        self.own_version = own_version
        self.done = False

    def wait(self):
        if not self.done:
            for *_, work in self.parts:
                work.wait()        # gloo: host wait; RCCL: the current stream waits
            if self.own[3] is not None:
                torch.cuda.current_stream().wait_event(self.own[3])
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
        # every rank creates every group in the same order (torch new_group rule)
        self.req = dist.new_group(list(range(self.world)), backend="gloo")
        # host barriers (resume) on a group of their own: the shard servers keep an
        # any-source receive posted on `req` at all times
        self.ctl = dist.new_group(list(range(self.world)), backend="gloo")
        backend = dist.get_backend(self.group)
        if self.cuda and backend != "nccl":
            raise RuntimeError("sharded_async with GPU payloads needs the RCCL ('nccl') "
                               "backend: gloo cannot move device tensors point-to-point")
        self.payload_backend = "rccl" if backend == "nccl" else "gloo"
        push, reply = make_p2p_groups(self.world, backend)
        pdev = self.device if backend == "nccl" else torch.device("cpu")
        warm_up_p2p(self.rank, push, pdev)
        warm_up_p2p(self.rank, reply, pdev)
        self.push_out = {k[1]: g for k, g in push.items() if k[0] == self.rank}
        self.reply_in = {k[0]: g for k, g in reply.items() if k[1] == self.rank}
        lo = self.rank * self.shard_n
        self.server = ShardServer(
            self.rank, self.world, self.arena.p32.detach()[lo: lo + self.shard_n], self.req,
            {k: g for k, g in push.items() if k[1] == self.rank},
            {k: g for k, g in reply.items() if k[0] == self.rank}, scale).start()
        self._pull_free: deque = deque()      # reusable reply staging sets (+ free event)
        self._push_work: list = [[], []]      # per hand-off slot: payload sends
        self.side = torch.cuda.Stream(self.device) if self.cuda else None
        if self.side is not None:
            warm_stream(self.side)     # bind its queue now, not mid-step

    def _bounds(self, o: int):
        return o * self.shard_n, (o + 1) * self.shard_n

    def push(self, step: int):
        slot = self._send_slot               # the hand-off slot _handoff fills next
        for w in self._push_work[slot]:      # that slot's previous sends are done
            w.wait()
        self._push_work[slot] = []
        buf = self._handoff()
        self._resolve_versions()
        for o in range(self.world):
            lo, hi = self._bounds(o)
            if o == self.rank:
                done = self.server.apply(buf[lo:hi], self.version)
                if done is not None:
                    # the PS stream reads this slot asynchronously (and may be
                    # parked in a slow peer's receive): the next hand-off into
                    # the slot, two pushes later, must wait for the apply
                    self._push_work[slot].append(_EventWork(done))
                continue
            header = M.make_header(M.MessageCode.GradientUpdate, self.rank, step, self.version,
                                   hi - lo, buf.dtype)
            M.SENDS.add(dist.isend(header, o, group=self.req, tag=M.TAG_HEADER), header)
            # RCCL: ordered after the hand-off kernel on the compute stream
            w = dist.isend(buf[lo:hi], o, group=self.push_out[o])
            self._push_work[slot].append(w if self.cuda else M.OnceWork(w))
        self.pushes += 1
        self.bytes_sent += buf.numel() * buf.element_size() * (self.world - 1) // self.world

    def request_pull(self, step: int):
        sn = self.shard_n
        free = self._pull_free.popleft() if len(self._pull_free) > self.staleness else None
        if free is None:
            # allocated on the side stream that receives into them (deterministic mode
            # NaN-fills torch.empty on the allocating stream); the own shard's snapshot
            # stream orders behind that too
            with (torch.cuda.stream(self.side) if self.cuda else _Null()):
                bufs = {o: torch.empty(sn + (0 if o == self.rank else 1), dtype=torch.float32,
                                       device=self.device) for o in range(self.world)}
            if self.cuda:
                self.server.stream.wait_stream(self.side)
            free_ev = None
        else:
            bufs, free_ev = free
        parts = []
        with (torch.cuda.stream(self.side) if self.cuda else _Null()):
            if free_ev is not None:
                self.side.wait_event(free_ev)        # the last land read these buffers
            for o in range(self.world):
                if o == self.rank:
                    continue
                lo, hi = self._bounds(o)
                header = M.make_header(M.MessageCode.ParameterRequest, self.rank, step, 0, 0)
                M.SENDS.add(dist.isend(header, o, group=self.req, tag=M.TAG_HEADER), header)
                work = dist.irecv(bufs[o], o, group=self.reply_in[o])
                parts.append((lo, hi, bufs[o], work if self.cuda else M.OnceWork(work)))
        lo, hi = self._bounds(self.rank)
        if self.cuda and free_ev is not None:
            self.server.stream.wait_event(free_ev)
        _, own_v, ev = self.server.snapshot(bufs[self.rank])
        self.pending.append(_Pending(step, bufs, work=_ShardedPull(
            parts, (lo, hi, bufs[self.rank], ev), own_v)))
        self.bytes_recv += self.arena.numel * 4 * (self.world - 1) // self.world

    def _land(self, pend):
        if self.debug_landing and self.in_compute:
            raise RuntimeError(
                f"pull of step {pend.step} landed inside a training step (between zero_grad "
                "and local_step): parameters would change under forward/backward")
        pull = pend.work
        pull.wait()
        arena = self.arena
        acc = self.opt.acc if self.pull_mode == "rebase" else None
        pieces = [(lo, hi, rbuf[: hi - lo]) for lo, hi, rbuf, _ in pull.parts]
        lo, hi, own, _ = pull.own
        pieces.append((lo, hi, own))
        with torch.no_grad():
            for lo, hi, src in pieces:
                if self.cuda:
                    self.nat.pull_land(arena.p32[lo:hi], src,
                                       acc[lo:hi] if acc is not None else None,
                                       arena.w16[lo:hi] if arena.w16 is not None else None)
                else:
                    arena.p32[lo:hi].copy_(src)
                    if acc is not None:
                        arena.p32[lo:hi].add_(acc[lo:hi])
            if not self.cuda and arena.w16 is not None:
                arena.w16.copy_(arena.p32)
        # per-shard versions in shard order (the own shard's is known on the host);
        # the landed base version is their MIN on every backend -- on GPU resolved
        # without a host sync once the copies' event has completed
        vsrcs = {lo // self.shard_n: rbuf[hi - lo:] for lo, hi, rbuf, _ in pull.parts}
        ov = pull.own_version
        vsrcs[self.rank] = ov if torch.is_tensor(ov) else torch.tensor([float(ov)])
        self._note_versions([vsrcs[o] for o in range(self.world)])
        ev = None
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record()            # the staging set is free once the land kernels ran
        self.pulls += 1
        arena.bump()
        self._pull_free.append((pend.buf, ev))

    def finish(self):
        super().finish()                       # lands every requested pull
        for lst in self._push_work:
            for w in lst:
                w.wait()
        for o in range(self.world):
            if o != self.rank:
                M.send_message(M.MessageCode.Shutdown, None, o, group=self.req)
        M.SENDS.drain()
        self.server.join()                     # returns once every rank has shut down
        if self.cuda:
            torch.cuda.current_stream().wait_stream(self.server.stream)

    def stats(self) -> dict:
        self._resolve_versions()
        st = super().stats()
        st["shard_versions"] = list(self.shard_versions)
        st.update(self.server.stats())
        st["payload"] = self.payload_backend
        return st

    @property
    def master(self) -> torch.Tensor:
        if self.cuda:
            self.server.stream.synchronize()
        return self.server.master

    def state_dict(self) -> dict:
        snap, v, ev = self.server.snapshot()
        if ev is not None:
            ev.synchronize()
        return {"kind": "sharded_async", "rank": self.rank, "world": self.world,
                "master": snap.detach().cpu(),
                "shard_version": int(v.item()) if torch.is_tensor(v) else int(v)}

    def load_state_dict(self, sd: dict):
        if sd.get("kind") != "sharded_async":
            return
        if sd["world"] != self.world or sd["rank"] != self.rank:
            raise ValueError(f"sharded PS checkpoint is for rank {sd['rank']}/{sd['world']}, "
                             f"this is rank {self.rank}/{self.world}")
        with self.server.lock:
            with self.server._ctx():
                self.server.master.copy_(sd["master"].to(self.server.device))
                self.server.applied.set(int(sd.get("shard_version", 0)))
            self.server.version = int(sd.get("shard_version", 0))
        if self.cuda:
            self.server.stream.synchronize()
        # every shard restored before anyone asks for it: without this barrier a
        # fast rank's forced pull could be answered with a peer's pre-restore shard
        dist.barrier(group=self.ctl)
        # re-sync the live parameters from every restored shard
        self.request_pull(0)
        self.land_due(0, force=True)
        self.arena.refresh_shadow()
