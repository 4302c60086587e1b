"""Central parameter server (reference C7: ``asgd.server.ParameterServer``).

Contract, reconstructed from /root/reference/example/main.py:135-138 and the
worker side /root/reference/asgd/optim/Asynchronous.py:34,49,59:
``ParameterServer(model=...)`` owns a flat fp32 shard; ``.run()`` serves

* ``ParameterUpdate``  -> initialise the shard from a worker's parameters,
* ``GradientUpdate``   -> ``shard += delta`` (delta already carries ``-lr``),
* ``ParameterRequest`` -> reply to the SENDER with the current shard,

until every worker has sent ``Shutdown`` (the reference's loop never ended,
SURVEY D9).  Additions: a version counter (number of applied deltas; pushes
report the version their base params came from, so the server measures
staleness), per-worker liveness, periodic checkpoints, and two payload paths:

* ``payload="gloo"`` - headers and payloads on the (CPU) gloo group;
* ``payload="rccl"`` - headers on a CPU gloo control group, payloads on a
  per-(PS, worker) RCCL communicator on the PS GPU.  The shard, the apply
  kernel and the reply snapshots stay on the GPU, and the links run
  concurrently (:mod:`.links`): every worker's receives and sends are posted
  on that worker's own stream and buffer ring, so transfers from different
  workers overlap (one xGMI link each).  Applies are COMPLETION-ordered: each
  worker's delta is added on that worker's own link stream right after its
  receive lands, with fp32 atomics (applies of different workers may overlap
  in time), so a slow worker's pending payload never delays
  another worker's apply.  A reply snapshot is taken on the requester's own
  stream: it observes that worker's own applies (read-your-writes) and
  whatever other workers' applies have landed by then -- the reference PS had
  no ordering between workers at all (/root/reference/example/main.py:135-138).
  No host syncs anywhere.
"""
from __future__ import annotations

import logging
import os
import queue
import threading
import time
from collections import Counter, defaultdict

import torch
import torch.distributed as dist

from . import messaging as M
from .arena import FlatArena
from .links import AppliedCount, PairGroupTransport, PairLinks, wait_on

_LOG = logging.getLogger(__name__)


def make_ps_groups(ps_rank: int = 0, payload: str = "gloo"):
    """Create the control group and per-pair payload groups.

    MUST be called by every rank, in the same order (torch ``new_group`` rule).
    Returns ``(control_group, {worker_rank: pair_group})``.
    """
    world = dist.get_world_size()
    backend = dist.get_backend()
    if payload == "gloo" and backend == "gloo":
        return None, {}
    ctrl = dist.new_group(list(range(world)), backend="gloo")
    pairs = {}
    for w in range(world):
        if w == ps_rank:
            continue
        pairs[w] = dist.new_group([min(ps_rank, w), max(ps_rank, w)],
                                  backend="nccl" if payload == "rccl" else "gloo")
    return ctrl, pairs


class ParameterServer:
    def __init__(self, model=None, numel: int | None = None, workers=None, control_group=None,
                 pair_groups=None, payload: str = "auto", device=None, init_policy: str = "first",
                 checkpoint_path: str | None = None, checkpoint_every: int = 0,
                 worker_timeout: float | None = None, delta_scale: str | float = "sum",
                 transport=None, trace_links: bool = False):
        """``delta_scale``: factor on every pushed delta -- ``"sum"`` (1.0, the
        reference Downpour PS: /root/reference/asgd/optim/Asynchronous.py:48-55
        ships raw accumulated updates that the PS adds), ``"mean"`` (1 / #workers:
        the W workers' concurrent deltas average instead of adding up, which keeps
        many-worker runs stable; profiles/ttl_n8_delta_scale_r2.txt), or a float."""
        if not dist.is_initialized():
            raise RuntimeError("ParameterServer needs torch.distributed to be initialised")
        self.rank = dist.get_rank()
        world = dist.get_world_size()
        self.workers = list(workers) if workers is not None else [
            r for r in range(world) if r != self.rank]
        if delta_scale == "sum":
            self.delta_scale = 1.0
        elif delta_scale == "mean":
            self.delta_scale = 1.0 / max(1, len(self.workers))
        else:
            self.delta_scale = float(delta_scale)
        if payload == "auto":
            payload = "rccl" if dist.get_backend() == "nccl" else "gloo"
        self.payload = payload
        self.ctrl = control_group
        self.pairs = pair_groups or {}
        self.links = None
        if payload == "rccl":
            if not self.pairs and transport is None:
                raise ValueError("payload='rccl' needs pair_groups from make_ps_groups()")
            self.device = torch.device(device or f"cuda:{torch.cuda.current_device()}")
            # ``transport``: the pair groups (RCCL) unless a test substitutes one
            self.links = PairLinks(self.device, transport or PairGroupTransport(self.pairs),
                                   trace=trace_links, peers=self.workers)
        else:
            self.device = torch.device(device or "cpu")
        if model is not None:
            # the wire layout is the workers' flat arena (64-aligned params,
            # channels_last 4-D weights, padded total), not the unpadded ravel
            flat = FlatArena(list(model.parameters()), device="cpu", shadow_dtype=None,
                             with_grads=False).p32
        elif numel is not None:
            flat = torch.zeros(numel, dtype=torch.float32)
        else:
            raise ValueError("ParameterServer needs a model or numel")
        self.numel = flat.numel()
        pad = (-self.numel) % 4
        self.shard = torch.zeros(self.numel + pad, dtype=torch.float32, device=self.device)
        self.shard[: self.numel].copy_(flat)
        self.version = 0
        self.initialized = False
        self.init_policy = init_policy
        self.counts: Counter = Counter()
        self.bytes_in = 0
        self.bytes_out = 0
        self.staleness: list[int] = []
        self.last_seen = {w: time.monotonic() for w in self.workers}
        self.worker_timeout = worker_timeout
        self.dropped: list[int] = []   # workers declared dead by the liveness check
        self.checkpoint_path = checkpoint_path
        self.checkpoint_every = checkpoint_every
        self._tracker = M.SendTracker()
        self._hq = None
        self._recv_bufs = defaultdict(dict)      # gloo payload path
        self._init_ev = None                     # last shard overwrite (device links)
        # link streams that read or write the shard (applies AND reply snapshots):
        # an overwrite (_set) orders behind all of them
        self._touched_on: set = set()
        self.stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        if self.links is not None:
            # every worker's payload rings up front (fp32 and bf16 wire), not at
            # the first transfer while other workers' transfers are in flight
            padded = self.numel + pad
            for w in self.workers:
                for dt in (torch.float32, torch.bfloat16):
                    self.links.reserve(w, self.numel, dt, alloc=padded)
                self.links.reserve(w, self.numel + 1, torch.float32, send=True)
            torch.cuda.synchronize(self.device)
        if self.device.type == "cuda":
            from ..ops._ext import native

            self._native = native()
        else:
            self._native = None
        # applies wholly landed: the version a reply is stamped with (links.AppliedCount);
        # self.version stays the host's ENQUEUE count (staleness of incoming pushes)
        self.applied = AppliedCount(self.device, self._native)
        if self.links is not None:
            self._warm_kernels(padded)

    def _warm_kernels(self, padded: int):
        """Launch every kernel of the apply / reply path once, before any transfer.
        HIP loads a kernel's code object at its first launch, and that load waited
        for the work in flight: the PS's first apply stalled every other link until
        the first receive had landed (tests/test_links_gpu.py).  A zero delta leaves
        the shard unchanged."""
        with torch.cuda.stream(self.stream):
            for dt in (torch.float32, torch.bfloat16):
                z = torch.zeros(padded, dtype=dt, device=self.device)
                self._native.ps_apply(self.shard, z, None, self.delta_scale)
                self._native.ps_apply(self.shard, z, None, self.delta_scale, True)
            snap = torch.empty(self.numel + 1, dtype=torch.float32, device=self.device)
            self._native.ps_count(self.applied.dev, 0)
            self._native.ps_stamp(self.applied.dev, snap[self.numel:])
            snap[: self.numel].copy_(self.shard[: self.numel])
        torch.cuda.synchronize(self.device)

    # -------------------------------------------------------------- payload io
    def _recv_payload(self, sender: int, nelem: int, dtype: torch.dtype):
        """Receive ``sender``'s payload -> ``(buf, ready_event, slot)``.

        Device path: posted on the sender's own link stream (:class:`PairLinks`);
        ``ready`` marks arrival, ``slot`` is released by the consumer.  gloo
        path: a blocking receive, ``ready`` and ``slot`` are ``None``."""
        if nelem != self.numel:
            raise RuntimeError(f"PS: worker {sender} sent {nelem} elements, the shard has "
                               f"{self.numel} (model/arena layout mismatch)")
        padded = nelem + ((-nelem) % 4)
        self.bytes_in += nelem * torch.empty(0, dtype=dtype).element_size()
        if self.links is not None:
            slot, ready = self.links.recv(sender, nelem, dtype, alloc=padded)
            return slot.buf, ready, slot
        bufs = self._recv_bufs[sender]
        buf = bufs.get(dtype)
        if buf is None or buf.numel() != padded:
            buf = torch.zeros(padded, dtype=dtype, device=self.device)
            bufs[dtype] = buf
        dist.recv(buf[:nelem], src=sender, group=self.ctrl, tag=M.TAG_PAYLOAD)
        return buf, None, None

    def _reply(self, dst: int):
        """ParameterUpdate to ``dst``: the shard followed by one fp32 element holding
        the PS version of the snapshot -- the number of applies it WHOLLY contains
        (:class:`.links.AppliedCount`: stamped on the device before the copy) --
        so the worker can report its staleness on its next push."""
        n = self.numel
        if self.links is not None:
            def fill(buf):
                self.applied.stamp(buf[n:])     # first: counts only landed applies
                buf[:n].copy_(self.shard[:n])   # snapshot: later applies never tear it

            # snapshot on dst's OWN link stream: behind dst's own applies (same
            # stream) and the last initialisation, never behind another worker's
            # payload still in flight
            s = self.links.stream(dst)
            with torch.cuda.stream(s):
                wait_on(s, self._init_ev)
            self._touched_on.add(dst)
            self.links.send(dst, n + 1, torch.float32, fill, s)
        else:
            snap = torch.empty(n + 1, dtype=torch.float32)
            snap[:n].copy_(self.shard[:n])
            self.applied.stamp(snap[n:])     # gloo: applies are synchronous
            w = dist.isend(snap, dst, group=self.ctrl, tag=M.TAG_REPLY)
            self._tracker.add(w, snap)
        self.bytes_out += (n + 1) * 4

    def _apply(self, delta: torch.Tensor, ready=None, slot=None, sender: int | None = None):
        """``shard += scale * delta``.  Device links: on the SENDER's link stream,
        right behind its receive (``ready`` is on that stream), with fp32 atomics
        so concurrent applies of different workers all land, releasing the receive
        ``slot`` when done.  Otherwise on the apply stream after ``ready``."""
        if self._native is not None and self.links is not None and sender is not None:
            s = self.links.stream(sender)
            with torch.cuda.stream(s):
                wait_on(s, ready)
                wait_on(s, self._init_ev)
                self._native.ps_apply(self.shard, delta, None, self.delta_scale, True)
                self.applied.bump()            # counted once this apply has landed
                if slot is not None:
                    self.links.release(slot, s)
            self._touched_on.add(sender)
        elif self._native is not None:
            with torch.cuda.stream(self.stream):
                wait_on(self.stream, ready)
                self._native.ps_apply(self.shard, delta, None, self.delta_scale)
                self.applied.bump()
                if slot is not None:
                    self.links.release(slot, self.stream)
        else:
            self.shard[: self.numel].add_(delta[: self.numel].to(torch.float32),
                                          alpha=self.delta_scale)
            self.applied.bump()
        self.version += 1

    def _set(self, params: torch.Tensor, ready=None, slot=None, version: int | None = None):
        with torch.cuda.stream(self.stream) if self.stream is not None else _null():
            wait_on(self.stream, ready)
            # an overwrite orders against every apply AND reply snapshot already
            # enqueued on a link (a reply in flight must not send a torn shard)
            for p in sorted(self._touched_on):
                ev = torch.cuda.Event()
                ev.record(self.links.stream(p))
                self.stream.wait_event(ev)
            self.shard[: self.numel].copy_(params[: self.numel])
            if version is not None:
                self.applied.set(version)   # the restored shard holds `version` applies
            if slot is not None:
                self.links.release(slot, self.stream)
            if self.links is not None:
                # later applies and reply snapshots (link streams) wait for it
                self._init_ev = torch.cuda.Event()
                self._init_ev.record(self.stream)

    # -------------------------------------------------------------------- loop
    def handle(self, code, sender: int, step: int, version: int, nelem: int, dtype):
        self.counts[code.name] += 1
        self.last_seen[sender] = time.monotonic()
        if code == M.MessageCode.GradientUpdate:
            delta, ready, slot = self._recv_payload(sender, nelem, dtype)
            self.staleness.append(self.version - version)
            self._apply(delta, ready, slot, sender)
            if self.checkpoint_every and self.version % self.checkpoint_every == 0:
                self.save_checkpoint()
        elif code == M.MessageCode.ParameterUpdate:
            params, ready, slot = self._recv_payload(sender, nelem, dtype)
            if not self.initialized or self.init_policy == "last":
                self._set(params, ready, slot)
                self.initialized = True
            elif slot is not None:
                slot.free = ready        # never read: free once it has arrived
        elif code == M.MessageCode.ParameterRequest:
            self._reply(sender)
        elif code == M.MessageCode.Checkpoint:
            self.save_checkpoint()
        elif code == M.MessageCode.Heartbeat:
            pass

    def _check_liveness(self, alive: set):
        if not self.worker_timeout:
            return
        now = time.monotonic()
        for w in list(alive):
            if now - self.last_seen[w] > self.worker_timeout:
                _LOG.warning("PS: worker %d silent for %.1fs, dropping", w,
                             now - self.last_seen[w])
                alive.discard(w)
                self.dropped.append(w)

    def _header_pump(self, q):
        """Receive thread: any-source headers into ``q`` until every worker has
        sent Shutdown.  Only headers (TAG_HEADER) are received here; payloads and
        replies use their own tags on the main thread."""
        remaining = set(self.workers)
        try:
            while remaining:
                hdr = M.recv_header(None, self.ctrl)
                q.put(hdr)
                if hdr[0] == M.MessageCode.Shutdown:
                    remaining.discard(hdr[1])
        except BaseException as e:   # surfaced to run()
            q.put(e)

    def _next_header(self, alive: set):
        """Any-source header receive.  With a ``worker_timeout`` headers arrive
        through a receive thread and the main loop waits on its queue with a
        timeout, so liveness is enforced even when NO message arrives (every
        remaining worker hung): returns ``None`` once nobody is left alive.
        (gloo work cannot be polled and a timed ``wait`` closes the connection.)"""
        if not self.worker_timeout:
            return M.recv_header(None, self.ctrl)
        if self._hq is None:
            self._hq = queue.Queue()
            threading.Thread(target=self._header_pump, args=(self._hq,), daemon=True,
                             name="ps-headers").start()
        tick = min(self.worker_timeout / 4, 0.5)
        while True:
            try:
                item = self._hq.get(timeout=tick)
            except queue.Empty:
                self._check_liveness(alive)
                if not alive:
                    return None
                continue
            if isinstance(item, BaseException):
                raise RuntimeError(f"PS header receive failed: {item!r}")
            return item

    def run(self):
        alive = set(self.workers)
        _LOG.info("PS rank %d serving workers %s (%s payload, %d params)", self.rank,
                  sorted(alive), self.payload, self.numel)
        while alive:
            try:
                hdr = self._next_header(alive)
            except RuntimeError as e:
                # A worker died (connection closed / timeout): keep what we have.
                _LOG.warning("PS: control receive failed (%r); stopping with %d live workers",
                             e, len(alive))
                break
            if hdr is None:
                break
            code, sender, step, version, nelem, dtype = hdr
            if code == M.MessageCode.Shutdown:
                alive.discard(sender)
                continue
            self.handle(code, sender, step, version, nelem, dtype)
            self._check_liveness(alive)
        self.finish()
        return self.stats()

    def finish(self):
        self._tracker.drain()
        self._sync_device()
        if self.checkpoint_path:
            self.save_checkpoint()

    def _sync_device(self):
        """Wait for every enqueued apply / overwrite / transfer (all streams)."""
        if self.links is not None:
            self.links.synchronize()
        if self.stream is not None:
            self.stream.synchronize()

    # --------------------------------------------------------------- utilities
    def parameters(self) -> torch.Tensor:
        self._sync_device()
        return self.shard[: self.numel]

    def stats(self) -> dict:
        st = self.staleness
        return {
            "version": self.version,
            "applied": self.applied.value(),
            "counts": dict(self.counts),
            "bytes_in": self.bytes_in,
            "bytes_out": self.bytes_out,
            "staleness_mean": (sum(st) / len(st)) if st else 0.0,
            "staleness_max": max(st) if st else 0,
            "dropped": list(self.dropped),
        }

    def save_checkpoint(self, path: str | None = None):
        path = path or self.checkpoint_path
        if not path:
            return
        from ..utils.checkpoint import save_ps_checkpoint

        save_ps_checkpoint(path, self.parameters().detach().cpu(), self.version, self.stats())

    def load_checkpoint(self, path: str):
        from ..utils.checkpoint import load_ps_checkpoint

        flat, version, _ = load_ps_checkpoint(path)
        self._set(flat.to(self.device), version=version)
        self.version = version
        self.initialized = True


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def serve(model=None, **kw):
    """Convenience: build a server for ``model`` and run it to completion."""
    return ParameterServer(model=model, **kw).run()


if os.environ.get("DMP_PS_DEBUG"):
    logging.basicConfig(level=logging.INFO)
