"""Link-concurrent payload path for parameter servers.

A PS GPU in the reference topology (1 PS + 7 workers on 8 GPUs) has one xGMI
link to every worker.  The reference's PS served all workers from one receive
loop (/root/reference/example/main.py:135-138; the worker side
/root/reference/asgd/optim/Asynchronous.py:34,49,59), and a straight port puts
every transfer on ONE stream: torch's RCCL p2p makes each operation's RCCL
stream wait on the current stream, so worker B's receive cannot start before
worker A's receive and apply have finished -- one link busy at a time.

:class:`PairLinks` gives every peer its own HIP stream and its own ring of
payload buffers:

* a receive from peer ``p`` is posted on ``stream[p]`` behind nothing but the
  apply that last read the ring slot it lands in, so receives from different
  peers are in flight at the same time (one link each);
* the consumer (the PS apply stream) waits on the receive's ``ready`` event
  and applies; :meth:`PairLinks.release` after the apply frees the slot;
* a reply is snapshotted on the apply stream (so it observes every apply
  enqueued before it) into the peer's send ring, then sent on ``stream[p]``.

The same code runs on CPU (gloo payloads, the multi-process tests): streams
are null contexts, a receive blocks the calling thread until it has arrived,
and a send slot is reused only after its previous send's ``Work`` completed.

The payload transport is pluggable: :class:`PairGroupTransport` is RCCL (one
2-rank communicator per pair, each with its own RCCL stream) or gloo, and a
test substitutes a delayed device copy with the same stream semantics
(``tests/test_links_gpu.py::test_ps_links_overlap_receives``).
"""
from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist

from .messaging import OnceWork


class PairGroupTransport:
    """Point-to-point payloads on one process group per peer (RCCL pair comms;
    ``groups[peer]`` carries every transfer to / from ``peer``)."""

    def __init__(self, groups: dict):
        self.groups = groups

    def irecv(self, buf: torch.Tensor, peer: int):
        return dist.irecv(buf, peer, group=self.groups[peer])

    def isend(self, buf: torch.Tensor, peer: int):
        return dist.isend(buf, peer, group=self.groups[peer])


class _HostEvent:
    """CPU stand-in for a stream event: complete once ``work`` (if any) is."""

    __slots__ = ("work",)

    def __init__(self, work=None):
        self.work = work

    def wait(self):
        if self.work is not None:
            self.work.wait()

    def query(self) -> bool:
        return self.work is None or self.work.is_completed()


_DONE = _HostEvent()


def wait_on(stream, ev):
    """Order ``stream`` after ``ev`` (GPU: a stream wait, the host never blocks;
    CPU: the calling thread waits for the host event)."""
    if ev is None:
        return
    if isinstance(ev, _HostEvent):
        ev.wait()
    else:
        stream.wait_event(ev)


def warm_stream(stream):
    """Submit one tiny kernel to a fresh HIP stream (binds its hardware queue
    while nothing is in flight; see :class:`PairLinks`)."""
    with torch.cuda.stream(stream):
        torch.zeros(1, device=stream.device)


class AppliedCount:
    """How many applies a PS shard has wholly received -- the version a reply is
    stamped with (the version is the basis of staleness-bounded
    pulls; the reference PS had none, /root/reference/asgd/optim/Asynchronous.py:
    17-18,48-59).

    With device links the applies run on several link streams at once, so a host
    counter bumped at ENQUEUE time overstates what a snapshot holds (a reply could
    carry only the requester's own deltas and say "version 4").  On GPU the count
    is a device int32: :meth:`bump` runs on the applying stream right after the
    apply kernel (it moves only once that apply has landed), :meth:`stamp` runs on
    the replying stream BEFORE the snapshot copy (``csrc/optim.hip`` ps_count /
    ps_stamp, agent-scope atomics).  A stamp therefore counts only applies the
    snapshot fully contains; applies in flight elsewhere may show up in some
    elements, never in the count.  On CPU applies are synchronous and the count
    is a host integer."""

    def __init__(self, device, native=None):
        self.cuda = device.type == "cuda"
        self.nat = native
        self.host = 0
        self.dev = torch.zeros(1, dtype=torch.int32, device=device) if self.cuda else None

    def bump(self):
        """One apply has been enqueued on the CURRENT stream (GPU: counted when it lands)."""
        self.host += 1
        if self.cuda:
            self.nat.ps_count(self.dev, 1)

    def set(self, value: int):
        """The shard was overwritten (init / checkpoint) on the current stream."""
        self.host = int(value)
        if self.cuda:
            self.nat.ps_count(self.dev, int(value), True)

    def stamp(self, dst: torch.Tensor):
        """Write the count into the 1-element fp32 ``dst`` on the current stream;
        call it BEFORE the snapshot copy."""
        if self.cuda:
            self.nat.ps_stamp(self.dev, dst.reshape(1))
        else:
            dst.fill_(float(self.host))

    def value(self) -> int:
        """Landed count (host sync on GPU: stats / checkpoints only)."""
        return int(self.dev.item()) if self.cuda else self.host


class _Slot:
    __slots__ = ("buf", "free", "work")

    def __init__(self, buf):
        self.buf = buf
        self.free = None     # event after which buf may be overwritten
        self.work = None     # keeps the last transfer's Work alive


class _Ring:
    __slots__ = ("slots", "i")

    def __init__(self):
        self.slots: list[_Slot] = []
        self.i = 0


class PairLinks:
    """Per-peer streams and buffer rings (see module docstring).

    ``depth`` buffers per (peer, direction, shape): a peer may have that many
    transfers of one kind in flight before a new one waits for the oldest.
    ``trace=True`` (GPU) records timing-event spans ``(kind, peer, start, end)``
    of every transfer in :attr:`spans` (tests, diagnostics)."""

    def __init__(self, device, transport, depth: int = 2, trace: bool = False, peers=()):
        """``peers``: create AND first-use their streams now.  The first
        submission to a fresh HIP stream blocked the host ~5 ms (its hardware
        queue is bound then): two peers' first transfers ran back to back with
        cold streams, overlapped with warmed ones.  Concurrency across peers also
        needs enough HIP hardware queues: at HIP's default of 4, two peers' link
        streams shared a queue and ran back to back; bench.py / launch.py give a
        PS process 16 (profiles/links_stream_creation_r4.txt)."""
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.transport = transport
        self.depth = max(1, depth)
        self.trace = trace and self.cuda
        self.spans: list = []
        self.counts = {"recv": 0, "send": 0, "reused": 0}
        self._streams: dict[int, torch.cuda.Stream] = {}
        self._rx: dict = {}
        self._tx: dict = {}
        for p in peers:
            self.stream(p)
        if self.cuda and self._streams:
            torch.cuda.synchronize(self.device)

    def stream(self, peer: int):
        if not self.cuda:
            return None
        s = self._streams.get(peer)
        if s is None:
            s = torch.cuda.Stream(self.device)
            self._streams[peer] = s
            warm_stream(s)
        return s

    def _ctx(self, stream):
        return torch.cuda.stream(stream) if self.cuda else contextlib.nullcontext()

    def reserve(self, peer: int, numel: int, dtype, alloc: int | None = None,
                send: bool = False):
        """Allocate ``peer``'s ring for payloads of this shape NOW: a first-use
        allocation in the middle of other peers' transfers can synchronise the
        device (like a stream creation)."""
        alloc = numel if alloc is None else alloc
        rings = self._tx if send else self._rx
        ring = rings.get((peer, alloc, dtype))
        if ring is None:
            ring = rings[(peer, alloc, dtype)] = _Ring()
        while len(ring.slots) < self.depth:
            ring.slots.append(_Slot(torch.zeros(alloc, dtype=dtype, device=self.device)))

    def _next(self, rings: dict, key, numel: int, dtype) -> _Slot:
        ring = rings.get(key)
        if ring is None:
            ring = rings[key] = _Ring()
        if len(ring.slots) < self.depth:
            # zero-filled: a padded tail (alloc > payload) stays zero forever
            slot = _Slot(torch.zeros(numel, dtype=dtype, device=self.device))
            ring.slots.append(slot)
            return slot
        slot = ring.slots[ring.i]
        ring.i = (ring.i + 1) % len(ring.slots)
        self.counts["reused"] += 1
        return slot

    def _event(self, stream=None, timing: bool = False):
        if not self.cuda:
            return _DONE
        ev = torch.cuda.Event(enable_timing=timing)
        ev.record(stream)
        return ev

    def recv(self, peer: int, numel: int, dtype, alloc: int | None = None):
        """Post a receive of ``numel`` elements from ``peer`` on the peer's stream
        (into the first ``numel`` of an ``alloc``-element, zero-padded buffer).

        Returns ``(slot, ready)``: ``slot.buf`` holds the payload once ``ready``
        has completed.  The caller MUST :meth:`release` the slot after its last
        read of ``slot.buf``."""
        alloc = numel if alloc is None else alloc
        slot = self._next(self._rx, (peer, alloc, dtype), alloc, dtype)
        s = self.stream(peer)
        self.counts["recv"] += 1
        with self._ctx(s):
            wait_on(s, slot.free)                # the apply that last read this slot
            start = self._event(s, True) if self.trace else None
            view = slot.buf if alloc == numel else slot.buf[:numel]
            slot.work = OnceWork(self.transport.irecv(view, peer)) if not self.cuda else \
                self.transport.irecv(view, peer)
            slot.work.wait()                     # GPU: a stream wait; CPU: arrival
            ready = self._event(s, self.trace)
        if self.trace:
            self.spans.append(("recv", peer, start, ready))
        return slot, ready

    def release(self, slot: _Slot, stream=None):
        """Mark ``slot`` reusable after the work enqueued so far on ``stream``."""
        slot.free = self._event(stream)
        return slot.free

    def send(self, peer: int, numel: int, dtype, fill, fill_stream) -> _Slot:
        """``fill(buf)`` on ``fill_stream`` (after the send that last used the
        slot completed), then send ``buf`` to ``peer`` on the peer's stream."""
        slot = self._next(self._tx, (peer, numel, dtype), numel, dtype)
        self.counts["send"] += 1
        with self._ctx(fill_stream):
            wait_on(fill_stream, slot.free)
            fill(slot.buf)
            filled = self._event(fill_stream)
        s = self.stream(peer)
        with self._ctx(s):
            wait_on(s, filled)
            start = self._event(s, True) if self.trace else None
            if self.cuda:
                slot.work = self.transport.isend(slot.buf, peer)
                slot.work.wait()
                slot.free = self._event(s, self.trace)
            else:
                # gloo reads the buffer when the peer's receive is posted: the slot
                # is free once that send has completed
                slot.work = OnceWork(self.transport.isend(slot.buf, peer))
                slot.free = _HostEvent(slot.work)
        if self.trace:
            self.spans.append(("send", peer, start, slot.free))
        return slot

    def synchronize(self):
        if self.cuda:
            for s in self._streams.values():
                s.synchronize()
            return
        for rings in (self._tx, self._rx):
            for ring in rings.values():
                for slot in ring.slots:
                    if slot.work is not None:
                        slot.work.wait()
