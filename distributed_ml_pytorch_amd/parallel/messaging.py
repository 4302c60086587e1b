"""Message protocol between workers and the parameter server (reference C9).

The reference imports ``MessageCode``, ``MessageListener`` and ``send_message``
from a module that does not exist upstream
(/root/reference/asgd/optim/Asynchronous.py:5; contract in SURVEY.md §2.2 C9).
This is the re-design:

* **Header / payload split.**  Every message is a small int64 header
  ``[code, sender, step, version, nelem, dtype]`` (tag ``TAG_HEADER``) followed,
  only when ``nelem > 0``, by a payload (tag ``TAG_PAYLOAD``).  A pull request
  carries NO payload (the reference sent a full-model dummy).
* **Any-source only on the header.**  The server receives headers from any
  sender, then receives the payload from that specific sender, so concurrent
  senders can never interleave payloads.  On GPU runs the header travels on a
  CPU gloo control group and the payload on a per-pair RCCL communicator
  (RCCL has no any-source receive and no tags).
* **Every send is tracked.**  The reference dropped the ``isend`` handles and
  lost messages on modern gloo (measured); :data:`SENDS` keeps each
  in-flight ``Work`` and its tensor alive until it completes.
"""
from __future__ import annotations

import enum
import logging
import threading
from collections import deque

import torch
import torch.distributed as dist

_LOG = logging.getLogger(__name__)

TAG_HEADER = 11
TAG_PAYLOAD = 12
TAG_REPLY = 13
HEADER_LEN = 6

_DTYPES = {0: torch.float32, 1: torch.bfloat16, 2: torch.float16}
_DTYPE_CODES = {v: k for k, v in _DTYPES.items()}


class MessageCode(enum.IntEnum):
    ParameterRequest = 0
    GradientUpdate = 1
    ParameterUpdate = 2
    Shutdown = 3
    Heartbeat = 4
    Checkpoint = 5


class OnceWork:
    """A ``Work`` whose ``wait()`` may be called any number of times.

    gloo's p2p ``Work`` reports ``is_completed() == False`` until ``wait()`` has
    been called, and a SECOND ``wait()`` on a completed send blocks forever
    (both measured on torch 2.10).  Every tracked send is wrapped, so the tracker
    and a client's buffer-reuse guard can both wait on it safely.
    """

    __slots__ = ("work", "done")

    def __init__(self, work):
        self.work = work
        self.done = False

    def wait(self):
        if not self.done:
            self.work.wait()
            self.done = True
        return True

    def is_completed(self) -> bool:
        return self.done or self.work.is_completed()


class SendTracker:
    """Keeps in-flight ``Work`` handles (and their buffers) alive until done.

    Completion cannot be polled on gloo (see :class:`OnceWork`), so the tracker
    is bounded instead: beyond ``max_inflight`` entries the oldest are waited
    for (long since received by then), which caps the payload memory it pins.
    """

    def __init__(self, max_inflight: int = 32):
        self._q: deque = deque()
        self._lock = threading.Lock()
        self.max_inflight = max_inflight

    def add(self, work, *keepalive):
        w = work if isinstance(work, OnceWork) else OnceWork(work)
        with self._lock:
            self._q.append((w, keepalive))
            self._reap_locked()
        while True:
            with self._lock:
                if len(self._q) <= self.max_inflight:
                    break
                old, _ = self._q.popleft()
            old.wait()
        return w

    def _reap_locked(self):
        while self._q and self._q[0][0].is_completed():
            self._q.popleft()

    def reap(self):
        with self._lock:
            self._reap_locked()

    def drain(self):
        while True:
            with self._lock:
                if not self._q:
                    return
                work, _ = self._q.popleft()
            work.wait()

    def __len__(self):
        return len(self._q)


SENDS = SendTracker()


def make_header(code, sender: int, step: int = 0, version: int = 0, nelem: int = 0,
                dtype: torch.dtype = torch.float32) -> torch.Tensor:
    return torch.tensor([int(code), sender, step, version, nelem, _DTYPE_CODES[dtype]],
                        dtype=torch.int64)


def parse_header(h: torch.Tensor):
    v = h.tolist()
    return MessageCode(v[0]), int(v[1]), int(v[2]), int(v[3]), int(v[4]), _DTYPES[int(v[5])]


def send_message(message_code, payload: torch.Tensor | None = None, dst: int = 0, step: int = 0,
                 version: int = 0, group=None, tracker: SendTracker | None = None):
    """Fire-and-track send of a header (+ payload) to ``dst`` (default: the PS, rank 0).

    Signature-compatible with the reference's ``send_message(code, payload)``
    call sites (Asynchronous.py:34,49,59); a ParameterRequest's payload is
    ignored (never sent).
    """
    tracker = tracker or SENDS
    rank = dist.get_rank()
    if message_code == MessageCode.ParameterRequest:
        payload = None
    nelem = 0 if payload is None else payload.numel()
    dt = torch.float32 if payload is None else payload.dtype
    header = make_header(message_code, rank, step, version, nelem, dt)
    works = [tracker.add(dist.isend(header, dst, group=group, tag=TAG_HEADER), header)]
    if nelem:
        buf = payload.detach().contiguous()
        works.append(tracker.add(dist.isend(buf, dst, group=group, tag=TAG_PAYLOAD), buf))
    return works


def recv_header(src: int | None = None, group=None):
    h = torch.empty(HEADER_LEN, dtype=torch.int64)
    dist.recv(h, src=src, group=group, tag=TAG_HEADER)
    return parse_header(h)


class MessageListener(threading.Thread):
    """Receive loop on its own thread, dispatching to :meth:`receive`.

    Same shape as the reference's base class (``MessageListener(model)``,
    ``.start()``, overridable ``receive(sender, message_code, parameter)``;
    Asynchronous.py:9-18,37-38).  Unlike the reference's Listener it never
    touches live parameters itself: subclasses hand payloads to a staging
    buffer and the optimizer swaps them in at a step boundary.
    """

    def __init__(self, model=None, numel: int | None = None, src: int | None = None, group=None):
        super().__init__(daemon=True)
        self.model = model
        if numel is None and model is not None:
            numel = sum(p.numel() for p in model.parameters())
        self.numel = numel or 0
        self.src = src
        self.group = group
        self._stop_evt = threading.Event()
        self.error: BaseException | None = None

    def receive(self, sender, message_code, parameter):  # pragma: no cover - abstract
        raise NotImplementedError

    def stop(self):
        self._stop_evt.set()

    def run(self):
        try:
            while not self._stop_evt.is_set():
                code, sender, step, version, nelem, dt = recv_header(self.src, self.group)
                payload = None
                if nelem:
                    payload = torch.empty(nelem, dtype=dt)
                    dist.recv(payload, src=sender, group=self.group, tag=TAG_PAYLOAD)
                if code == MessageCode.Shutdown:
                    break
                _LOG.info("listener: %s from %d (step %d)", code.name, sender, step)
                self.receive(sender, code, payload)
        except BaseException as e:  # surfaced to the owner via .error
            self.error = e
            _LOG.warning("listener stopped: %r", e)
