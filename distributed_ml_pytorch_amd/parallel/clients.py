"""Worker-side parameter-server clients for the Downpour/ASGD optimizer.

One interface, four transports:

* :class:`LocalPSClient`   - in-process PS on the worker's own device (1 GPU).
* :class:`GlooPSClient`    - the reference topology: rank ``ps_rank`` runs
  :class:`~.server.ParameterServer`, headers+payloads over gloo (CPU tensors).
* :class:`RcclPSClient`    - same topology on GPUs: header on a CPU gloo control
  group, payload on a per-(PS, worker) RCCL communicator (xGMI link).
* :class:`ShardedPSClient` - DistBelief-style sharded PS co-located on every
  worker: a push is a reduce-scatter of the accumulated deltas into each
  rank's fp32 master shard (+ apply), a pull is an all-gather of the shards.
  On 8 GPUs this drives all 7 xGMI links of every GPU instead of funnelling
  through one PS GPU.

Timing semantics shared by all clients (``staleness = s``):
  step k:   fused update -> [push if k % n_push == 0] -> [pull request if
            k % n_pull == 0] -> land every pull requested at step <= k - s.
On GPU, push/pull communication runs on a side stream / the RCCL stream and a
pull is landed by making the compute stream wait on its event, so the host
never blocks and forward/backward of steps k+1..k+s overlap the transfer.
"""
from __future__ import annotations

import logging
import os
from collections import deque

import torch
import torch.distributed as dist

from . import messaging as M
from .links import warm_stream

_LOG = logging.getLogger(__name__)


class _Pending:
    __slots__ = ("step", "buf", "work", "event", "version", "vsrc")

    def __init__(self, step, buf, work=None, event=None, version=0, vsrc=None):
        self.step, self.buf, self.work, self.event, self.version = step, buf, work, event, version
        # central PS replies carry the PS version as one trailing fp32 element
        self.vsrc = vsrc


class PSClient:
    """Base class: owns staging buffers and the landing logic."""

    def __init__(self, staleness: int = 1, pull_mode: str = "overwrite",
                 wire_dtype: torch.dtype = torch.float32):
        if staleness < 0:
            raise ValueError("staleness must be >= 0")
        if pull_mode not in ("overwrite", "rebase"):
            raise ValueError("pull_mode must be 'overwrite' (reference) or 'rebase'")
        self.staleness = staleness
        self.pull_mode = pull_mode
        self.wire_dtype = wire_dtype
        self.pending: deque[_Pending] = deque()
        self.version = 0            # version of the PS params last landed
        self.pushes = 0
        self.pulls = 0
        self.bytes_sent = 0
        self.bytes_recv = 0
        # SURVEY §5.2 debug check: a pulled snapshot may only land between steps
        # (the reference's listener thread overwrote parameters mid-step).  The
        # optimizer flags the compute half of a step (zero_grad .. local_step);
        # DMP_DEBUG_LANDING=1 turns a landing inside it into an error.
        self.debug_landing = os.environ.get("DMP_DEBUG_LANDING", "0") == "1"
        self.in_compute = False

    # -- wiring ------------------------------------------------------------
    def attach(self, opt):
        self.opt = opt
        self.arena = opt.arena
        self.device = self.arena.device
        self.cuda = self.device.type == "cuda"
        if self.cuda:
            from ..ops._ext import native

            self.nat = native()
        self._send = [None, None]
        self._send_work = [None, None]
        self._send_slot = 0

    def init(self):
        pass

    # -- push --------------------------------------------------------------
    def _handoff(self, n: int | None = None) -> torch.Tensor:
        """Snapshot the accumulator into a send buffer and zero it."""
        acc = self.opt.acc
        slot = self._send_slot
        self._send_slot ^= 1
        prev = self._send_work[slot]
        if prev is not None:
            prev.wait()
            self._send_work[slot] = None
        buf = self._send[slot]
        if buf is None or buf.numel() != acc.numel():
            buf = torch.empty(acc.numel(), dtype=self.wire_dtype, device=self.device)
            self._send[slot] = buf
        if self.cuda:
            if self.wire_dtype == torch.float32:
                self.nat.push_handoff(acc, buf, None)
            else:
                self.nat.push_handoff(acc, None, buf)
        else:
            buf.copy_(acc)
            acc.zero_()
        self._cur_slot = slot
        return buf

    def push(self, step: int):
        raise NotImplementedError

    def request_pull(self, step: int):
        raise NotImplementedError

    # -- landing -----------------------------------------------------------
    def _land(self, pend: _Pending):
        if self.debug_landing and self.in_compute:
            raise RuntimeError(
                f"pull of step {pend.step} landed inside a training step (between zero_grad "
                "and local_step): parameters would change under forward/backward")
        arena = self.arena
        acc = self.opt.acc if self.pull_mode == "rebase" else None
        src = pend.buf
        if self.cuda:
            if pend.event is not None:
                torch.cuda.current_stream().wait_event(pend.event)
            if pend.work is not None:
                pend.work.wait()
            n = arena.numel
            self.nat.pull_land(arena.p32, src[:n] if src.numel() != n else src,
                               acc, arena.w16)
        else:
            if pend.work is not None:
                pend.work.wait()
            with torch.no_grad():
                n = arena.numel
                flat = src[:n].to(torch.float32) if src.numel() >= n else None
                if flat is None:
                    arena.p32.zero_()
                    arena.p32[: src.numel()].copy_(src)
                else:
                    arena.p32.copy_(flat)
                if acc is not None:
                    arena.p32.add_(acc)
                if arena.w16 is not None:
                    arena.w16.copy_(arena.p32)
        self.version = max(self.version, pend.version)
        if pend.vsrc is not None:
            self._note_version(pend.vsrc)
        self.pulls += 1
        arena.bump()

    def _note_version(self, vsrc: torch.Tensor):
        """Record the PS version a landed reply was taken at, without a host sync
        on GPU (pinned async copy, read once its event has completed)."""
        if vsrc.device.type == "cpu":
            self.version = max(self.version, int(vsrc.item()))
            return
        if not hasattr(self, "_vq"):
            self._vq = deque()
        host = torch.empty(1, dtype=torch.float32, pin_memory=True)
        host.copy_(vsrc.reshape(1), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._vq.append((host, ev, False))

    def _note_versions(self, vsrcs: list):
        """Versions of the shards of ONE landed pull (shard order): recorded as
        :attr:`shard_versions`, and the landed base version is their minimum.
        Device sources are copied to pinned memory and resolved once their
        event has completed (no host sync); host sources resolve at once."""
        if all(v.device.type == "cpu" for v in vsrcs):
            self._set_shard_versions([int(v.reshape(-1)[0].item()) for v in vsrcs])
            return
        if not hasattr(self, "_vq"):
            self._vq = deque()
        host = torch.empty(len(vsrcs), dtype=torch.float32, pin_memory=True)
        for i, v in enumerate(vsrcs):
            host[i:i + 1].copy_(v.reshape(1), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._vq.append((host, ev, True))

    def _set_shard_versions(self, vals: list):
        self.shard_versions = vals
        if vals:
            self.version = max(self.version, min(vals))

    def _resolve_versions(self):
        vq = getattr(self, "_vq", None)
        while vq and vq[0][1].query():
            host, _, group = vq.popleft()
            if group:
                self._set_shard_versions([int(x) for x in host.tolist()])
            else:
                self.version = max(self.version, int(host.item()))

    def land_due(self, step: int, force: bool = False):
        while self.pending and (force or self.pending[0].step <= step - self.staleness):
            self._land(self.pending.popleft())

    def finish(self):
        self.land_due(0, force=True)
        for w in self._send_work:
            if w is not None:
                w.wait()
        M.SENDS.drain()

    def stats(self) -> dict:
        st = {"pushes": self.pushes, "pulls": self.pulls, "bytes_sent": self.bytes_sent,
              "bytes_recv": self.bytes_recv, "version": self.version}
        st.update(self.comm_times())
        return st

    # -- device-side timing of the communication (side stream) --------------
    def _timed(self, kind: str):
        """Context recording start/end events on the CURRENT stream around a
        communication phase; resolved lazily by :meth:`comm_times` (no sync)."""
        return _EventSpan(self, kind) if self.cuda else _NULL_SPAN

    def comm_times(self) -> dict:
        spans = getattr(self, "_spans", None)
        if not spans:
            return {}
        out = {}
        for kind, evs in spans.items():
            ms = [a.elapsed_time(b) for a, b in evs if b.query()]
            if ms:
                out[f"{kind}_device_ms"] = round(sum(ms) / len(ms), 4)
        return out

    # -- checkpoint state of the PS side held by this client ----------------
    def state_dict(self) -> dict:
        return {}

    def load_state_dict(self, sd: dict):
        pass


class LocalPSClient(PSClient):
    """In-process parameter server on the worker's device (single-GPU / tests).

    With ``DMP_LOCAL_PS_SIDE=1`` the PS work runs on the side HIP stream, ordered by
    events exactly as the
    N > 1 clients order theirs (:class:`ShardedPSClient` push / pull): the
    compute stream only hands the accumulator off (``push_handoff``); the
    master's apply and the pull snapshot run on ``side`` behind that event and
    overlap the next step's forward, and a pulled snapshot lands on the compute
    stream behind the snapshot's event at the staleness-bounded step boundary.
    So the 1-GPU headline exercises the same overlap structure as the
    multi-GPU topologies (BASELINE north star: "param pulls overlapped with
    forward on a side HIP stream"), and reports its ``push`` / ``pull`` device
    spans (``comm_times``)."""

    # Measured slower on the 1-GPU bench (same box, alternating runs: 3.68-3.69 vs
    # 3.615-3.617 ms per ResNet-18 step, profiles/local_ps_side_stream_r6.txt), so the
    # default keeps the apply and the snapshot on the compute stream; DMP_LOCAL_PS_SIDE=1
    # selects the side-stream placement described above (the N > 1 structure).
    SIDE = os.environ.get("DMP_LOCAL_PS_SIDE", "0") == "1"

    def init(self):
        self.master = self.arena.p32.detach().clone()
        self.ps_version = 0
        self.side = torch.cuda.Stream(self.device) if self.cuda else None
        self._pull_bufs: deque = deque()       # (snapshot buffer, land-done event)
        if self.cuda and not self.SIDE:
            self.side = torch.cuda.current_stream(self.device)
        if self.side is not None:
            warm_stream(self.side)     # bind its queue now, not mid-step
            # the master copy above was made on the compute stream
            self.side.wait_stream(torch.cuda.current_stream(self.device))

    def push(self, step: int):
        buf = self._handoff()
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record()                          # the hand-off kernel wrote buf
            with torch.cuda.stream(self.side):
                self.side.wait_event(ev)
                with self._timed("push"):
                    self.nat.ps_apply(self.master, buf, None, 1.0)
                done = torch.cuda.Event()
                done.record()
            # the hand-off slot is refilled two pushes later: after this apply read it
            self._send_work[self._cur_slot] = _EventWork(done)
        else:
            self.master.add_(buf.to(torch.float32))
        self.ps_version += 1
        self.pushes += 1
        self.bytes_sent += buf.numel() * buf.element_size()

    def request_pull(self, step: int):
        if not self.cuda:
            snap = self.master.clone() if self.wire_dtype == torch.float32 else \
                self.master.to(self.wire_dtype)
            self.pending.append(_Pending(step, snap, version=self.ps_version))
            self.bytes_recv += snap.numel() * snap.element_size()
            return
        with torch.cuda.stream(self.side):
            # allocated ON the side stream: anything the allocator does to a new block
            # (deterministic mode NaN-fills torch.empty) is ordered before the copy
            buf, free_ev = self._pull_bufs.popleft() if len(self._pull_bufs) > self.staleness \
                else (torch.empty(self.master.numel(), dtype=self.wire_dtype,
                                  device=self.device), None)
            if free_ev is not None:
                self.side.wait_event(free_ev)   # the land kernel that last read buf is done
            with self._timed("pull"):
                buf.copy_(self.master)          # behind every apply enqueued on `side`
            ev = torch.cuda.Event()
            ev.record()
        self.pending.append(_Pending(step, buf, event=ev, version=self.ps_version))
        self.bytes_recv += buf.numel() * buf.element_size()

    def _land(self, pend):
        super()._land(pend)
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record()              # side may refill the buffer after the land kernel
            self._pull_bufs.append((pend.buf, ev))

    def finish(self):
        super().finish()
        if self.cuda:
            self.side.synchronize()

    def state_dict(self) -> dict:
        if self.cuda:
            self.side.synchronize()
        return {"kind": "local", "master": self.master.detach().cpu(),
                "ps_version": int(self.ps_version)}

    def load_state_dict(self, sd: dict):
        if sd.get("kind") != "local":
            return
        if self.cuda:
            torch.cuda.current_stream().wait_stream(self.side)
        with torch.no_grad():
            self.master.copy_(sd["master"].to(self.master.device))
        if self.cuda:
            self.side.wait_stream(torch.cuda.current_stream())
        self.ps_version = int(sd["ps_version"])


class SharedPS:
    """One fp32 master vector served to several in-process workers.

    Backs the "virtual workers" mode: K model replicas in ONE
    process on one GPU, each stepping on its own HIP stream, all pushing to and
    pulling from this master - the reference's 1 PS + N workers topology
    (``Makefile:13-20``) without a second device.  Every apply and snapshot runs
    on the PS's own stream, so concurrent pushes from different worker streams
    are serialised exactly as the central PS serialises its receive loop, and a
    pull observes every push enqueued before it.
    """

    def __init__(self):
        self.master = None
        self.version = 0
        self.stream = None
        self.nat = None

    def adopt_or_set(self, p32: torch.Tensor) -> bool:
        """First caller seeds the master (the worker's init ParameterUpdate,
        ``Asynchronous.py:34``); later callers get ``False`` and copy it."""
        if self.master is not None:
            return False
        self.master = p32.detach().to(torch.float32).clone()
        if self.master.device.type == "cuda":
            from ..ops._ext import native

            self.nat = native()
            self.stream = torch.cuda.Stream(self.master.device)
            self.stream.wait_stream(torch.cuda.current_stream())
        return True

    def apply(self, delta: torch.Tensor):
        """``master += delta`` after the caller's stream reaches this point;
        returns the event marking the apply done (``None`` on CPU)."""
        self.version += 1
        if self.stream is None:
            self.master.add_(delta.to(torch.float32))
            return None
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream):
            self.nat.ps_apply(self.master, delta, None, 1.0)
            done = torch.cuda.Event()
            done.record()
        return done

    def snapshot(self, wire_dtype: torch.dtype):
        """Copy of the master as of every apply enqueued so far -> (buf, event)."""
        if self.stream is None:
            return self.master.clone() if wire_dtype == torch.float32 else \
                self.master.to(wire_dtype), None
        caller = torch.cuda.current_stream()
        with torch.cuda.stream(self.stream):
            buf = self.master.clone() if wire_dtype == torch.float32 else \
                self.master.to(wire_dtype)
            ev = torch.cuda.Event()
            ev.record()
        buf.record_stream(caller)    # landed (read) on the worker's stream
        return buf, ev


class SharedPSClient(PSClient):
    """Worker side of :class:`SharedPS` (virtual workers on one device)."""

    def __init__(self, shared: SharedPS, **kw):
        super().__init__(**kw)
        self.shared = shared

    def init(self):
        if not self.shared.adopt_or_set(self.arena.p32):
            if self.shared.stream is not None:
                torch.cuda.current_stream().wait_stream(self.shared.stream)
            with torch.no_grad():
                self.arena.p32.copy_(self.shared.master)
            self.arena.refresh_shadow()

    def push(self, step: int):
        buf = self._handoff()
        done = self.shared.apply(buf)
        if done is not None:
            # the send buffer is reused two pushes later: wait for this apply first
            self._send_work[self._cur_slot] = _EventWork(done)
        self.pushes += 1
        self.bytes_sent += buf.numel() * buf.element_size()

    def request_pull(self, step: int):
        buf, ev = self.shared.snapshot(self.wire_dtype)
        self.pending.append(_Pending(step, buf, event=ev, version=self.shared.version))
        self.bytes_recv += buf.numel() * buf.element_size()


class GlooPSClient(PSClient):
    """Reference topology over gloo: ``send_message`` to the PS, reply on TAG_REPLY."""

    def __init__(self, ps_rank: int = 0, group=None, **kw):
        super().__init__(**kw)
        self.ps_rank = ps_rank
        self.group = group

    def _cpu(self, t):
        return t if t.device.type == "cpu" else t.cpu()

    def init(self):
        self.used = self.arena.numel
        # a snapshot: gloo reads a CPU send buffer only when the PS posts its receive,
        # by which time the local steps may have moved the live parameters
        snap = self.arena.p32.detach().clone() if not self.cuda else self._cpu(self.arena.p32)
        M.send_message(M.MessageCode.ParameterUpdate, snap, self.ps_rank, step=0,
                       group=self.group)

    def push(self, step: int):
        buf = self._handoff()
        self._resolve_versions()
        works = M.send_message(M.MessageCode.GradientUpdate, self._cpu(buf), self.ps_rank,
                               step=step, version=self.version, group=self.group)
        if not self.cuda:
            # gloo reads an unbound CPU send buffer only when the PS posts its recv:
            # the slot must not be refilled (two pushes later) before that happens
            self._send_work[self._cur_slot] = works[-1]
        self.pushes += 1
        self.bytes_sent += buf.numel() * buf.element_size()

    def request_pull(self, step: int):
        M.send_message(M.MessageCode.ParameterRequest, None, self.ps_rank, step=step,
                       group=self.group)
        n = self.arena.numel
        buf = torch.empty(n + 1, dtype=torch.float32)
        work = dist.irecv(buf, self.ps_rank, group=self.group, tag=M.TAG_REPLY)
        self.pending.append(_Pending(step, buf, work=M.OnceWork(work), vsrc=buf[n]))
        self.bytes_recv += buf.numel() * 4

    def _land(self, pend):
        if self.cuda:
            pend.work.wait()
            pend.work = None
            n = self.arena.numel
            self.version = max(self.version, int(pend.buf[n].item()))
            pend.vsrc = None
            pend.buf = pend.buf[:n].to(self.device, non_blocking=False)
        super()._land(pend)

    def finish(self):
        super().finish()
        M.send_message(M.MessageCode.Shutdown, None, self.ps_rank, group=self.group)
        M.SENDS.drain()


class RcclPSClient(PSClient):
    """Central PS on GPUs: control header on gloo, payload over a per-pair RCCL comm."""

    def __init__(self, ps_rank: int, control_group, pair_group, **kw):
        super().__init__(**kw)
        self.ps_rank = ps_rank
        self.ctrl = control_group
        self.pair = pair_group
        self._pull_bufs: deque = deque()

    def _send_payload(self, buf):
        # torch's RCCL p2p waits on the current (compute) stream, so the send is
        # ordered after the hand-off kernel without a host sync.
        return dist.isend(buf, self.ps_rank, group=self.pair)

    def init(self):
        n = self.arena.numel
        header = M.make_header(M.MessageCode.ParameterUpdate, dist.get_rank(), 0, 0, n)
        M.SENDS.add(dist.isend(header, self.ps_rank, group=self.ctrl, tag=M.TAG_HEADER), header)
        w = self._send_payload(self.arena.p32)
        w.wait()

    def push(self, step: int):
        buf = self._handoff()
        self._resolve_versions()
        header = M.make_header(M.MessageCode.GradientUpdate, dist.get_rank(), step, self.version,
                               buf.numel(), buf.dtype)
        M.SENDS.add(dist.isend(header, self.ps_rank, group=self.ctrl, tag=M.TAG_HEADER), header)
        self._send_work[self._cur_slot] = self._send_payload(buf)
        self.pushes += 1
        self.bytes_sent += buf.numel() * buf.element_size()

    def request_pull(self, step: int):
        header = M.make_header(M.MessageCode.ParameterRequest, dist.get_rank(), step, 0, 0)
        M.SENDS.add(dist.isend(header, self.ps_rank, group=self.ctrl, tag=M.TAG_HEADER), header)
        n = self.arena.numel
        buf = self._pull_bufs.popleft() if len(self._pull_bufs) > self.staleness else \
            torch.empty(n + 1, dtype=torch.float32, device=self.device)
        work = dist.irecv(buf, self.ps_rank, group=self.pair)
        self.pending.append(_Pending(step, buf, work=work, vsrc=buf[n]))
        self.bytes_recv += buf.numel() * 4

    def _land(self, pend):
        super()._land(pend)
        self._pull_bufs.append(pend.buf)

    def finish(self):
        super().finish()
        header = M.make_header(M.MessageCode.Shutdown, dist.get_rank(), 0, 0, 0)
        dist.send(header, self.ps_rank, group=self.ctrl, tag=M.TAG_HEADER)
        M.SENDS.drain()


class ShardedPSClient(PSClient):
    """Sharded PS co-located on every worker (collective push/pull).

    Each rank owns ``numel / world`` of the fp32 master parameters.  Push =
    ``reduce_scatter(sum of every worker's accumulated delta)`` + apply into the
    local master shard (exactly what a central PS does for simultaneous
    pushes); pull = ``all_gather`` of the master shards.  On GPU both run on a
    side stream; the pull's event is waited by the compute stream only when
    the pull is due (``staleness`` steps later).
    """

    def __init__(self, group=None, force_collectives: bool = False, delta_scale: str | float = "sum",
                 **kw):
        """``delta_scale``: how the W simultaneous pushes combine in the master.
        ``"sum"`` (default) is what a central Downpour PS does - it adds every
        worker's delta (/root/reference/asgd/optim/Asynchronous.py:58-59, SURVEY
        C7) - so the effective step grows with W; ``"mean"`` scales the summed
        delta by 1/W (model averaging); a float is used as is."""
        super().__init__(**kw)
        self.group = group
        # run the RCCL path even at world size 1 (single-GPU validation)
        self.force = force_collectives
        self.delta_scale = delta_scale

    def init(self):
        self.world = dist.get_world_size(self.group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(self.group) if dist.is_initialized() else 0
        n = self.arena.numel
        if n % self.world:
            raise ValueError(f"arena length {n} not divisible by world size {self.world}")
        self.shard_n = n // self.world
        if self.delta_scale == "sum":
            self.scale = 1.0
        elif self.delta_scale == "mean":
            self.scale = 1.0 / self.world
        else:
            self.scale = float(self.delta_scale)
        if self.world > 1 or self.force:
            # identical starting point everywhere (the reference let every worker
            # start from its own random init and converge through pulls)
            dist.broadcast(self.arena.p32, 0, group=self.group)
            self.arena.refresh_shadow()
        lo = self.rank * self.shard_n
        self.master = self.arena.p32[lo: lo + self.shard_n].detach().clone()
        # fp32 wire: reduce-scatter the deltas (fp32 sums on the wire).  bf16 wire:
        # an all-to-all moves the same (W-1)/W of the bytes, but every rank gets
        # the W bf16 slices of its shard unreduced and adds them to its fp32
        # master one by one -- no bf16 partial sums (a bf16 reduce-scatter would
        # round the running sum to 8 bits at every hop of the ring)
        self.bf16_wire = self.wire_dtype == torch.bfloat16
        if self.bf16_wire:
            self.delta_slices = torch.zeros(self.world * self.shard_n, dtype=torch.bfloat16,
                                            device=self.device)
            self.master16 = torch.zeros(self.shard_n, dtype=torch.bfloat16, device=self.device)
        else:
            self.delta_shard = torch.zeros(self.shard_n, dtype=self.wire_dtype,
                                           device=self.device)
        self.side = torch.cuda.Stream(self.device) if self.cuda else None
        if self.side is not None:
            warm_stream(self.side)     # bind its queue now, not mid-step
        self._pull_bufs: deque = deque()
        self._push_event = None

    def _apply_delta(self):
        if self.bf16_wire:
            sn = self.shard_n
            for k in range(self.world):            # fp32 accumulation, one slice at a time
                sl = self.delta_slices[k * sn:(k + 1) * sn]
                if self.cuda:
                    self.nat.ps_apply(self.master, sl, None, self.scale)
                else:
                    self.master.add_(sl.to(torch.float32), alpha=self.scale)
        elif self.cuda:
            self.nat.ps_apply(self.master, self.delta_shard, None, self.scale)
        else:
            self.master.add_(self.delta_shard.to(torch.float32), alpha=self.scale)

    def _exchange_deltas(self, buf, async_op: bool):
        """Deltas of every rank for this rank's shard: reduce-scatter (fp32 wire)
        or all-to-all of the bf16 slices (bf16 wire)."""
        gloo = dist.get_backend(self.group) == "gloo"
        if self.bf16_wire:
            if gloo:
                dist.all_to_all_single(self.delta_slices, buf, group=self.group)
                return None
            return dist.all_to_all_single(self.delta_slices, buf, group=self.group,
                                          async_op=async_op)
        if gloo:
            self._gloo_reduce_scatter(buf)
            return None
        return dist.reduce_scatter_tensor(self.delta_shard, buf, group=self.group,
                                          async_op=async_op)

    def push(self, step: int):
        buf = self._handoff()
        self.pushes += 1
        self.bytes_sent += buf.numel() * buf.element_size() * (self.world - 1) // max(self.world, 1)
        if self.world == 1 and not self.force:
            if self.cuda:
                self.nat.ps_apply(self.master, buf, None, 1.0)
            else:
                self.master.add_(buf.to(torch.float32))
            return
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record()
            with torch.cuda.stream(self.side):
                self.side.wait_event(ev)
                with self._timed("push"):
                    work = self._exchange_deltas(buf, async_op=True)
                    if work is not None:
                        work.wait()
                    self._apply_delta()
                done = torch.cuda.Event()
                done.record()
            self._send_work[self._cur_slot] = _EventWork(done)
        else:
            self._exchange_deltas(buf, async_op=False)
            self._apply_delta()

    def _gloo_reduce_scatter(self, buf):
        # gloo has no reduce_scatter_tensor: all_reduce the flat buffer, keep our shard.
        tmp = buf.clone()
        dist.all_reduce(tmp, group=self.group)
        lo = self.rank * self.shard_n
        self.delta_shard.copy_(tmp[lo: lo + self.shard_n])

    def request_pull(self, step: int):
        n = self.arena.numel
        wdt = torch.bfloat16 if self.bf16_wire else torch.float32
        if self.cuda and (self.world > 1 or self.force):
            with torch.cuda.stream(self.side):
                # allocated on the side stream that fills it (see LocalPSClient)
                buf, free_ev = self._pull_bufs.popleft() \
                    if len(self._pull_bufs) > self.staleness else \
                    (torch.empty(n, dtype=wdt, device=self.device), None)
        else:
            buf, free_ev = self._pull_bufs.popleft() \
                if len(self._pull_bufs) > self.staleness else \
                (torch.empty(n, dtype=wdt, device=self.device), None)
        self.bytes_recv += n * buf.element_size() * (self.world - 1) // max(self.world, 1)
        if self.world == 1 and not self.force:
            buf.copy_(self.master)
            self.pending.append(_Pending(step, buf))
            return
        if self.cuda:
            with torch.cuda.stream(self.side):
                if free_ev is not None:
                    self.side.wait_event(free_ev)   # previous land kernel done reading buf
                with self._timed("pull"):
                    src = self.master
                    if self.bf16_wire:
                        self.master16.copy_(self.master)    # RNE cast on the side stream
                        src = self.master16
                    work = dist.all_gather_into_tensor(buf, src, group=self.group,
                                                       async_op=True)
                    work.wait()
                ev = torch.cuda.Event()
                ev.record()
            self.pending.append(_Pending(step, buf, event=ev))
        else:
            src = self.master
            if self.bf16_wire:
                self.master16.copy_(self.master)
                src = self.master16
            work = dist.all_gather_into_tensor(buf, src, group=self.group, async_op=True) \
                if dist.get_backend(self.group) != "gloo" else self._gloo_all_gather(buf, src)
            self.pending.append(_Pending(step, buf, work=work))

    def _gloo_all_gather(self, buf, src=None):
        src = self.master if src is None else src
        chunks = list(buf.view(self.world, self.shard_n).unbind(0))
        return dist.all_gather(chunks, src.contiguous(), group=self.group, async_op=True)

    def _land(self, pend):
        super()._land(pend)
        ev = None
        if self.cuda:
            # the buffer may be re-used by the side stream only after the land kernel
            ev = torch.cuda.Event()
            ev.record()
        self._pull_bufs.append((pend.buf, ev))

    def finish(self):
        super().finish()
        if self.cuda:
            self.side.synchronize()

    def state_dict(self) -> dict:
        if self.cuda:
            self.side.synchronize()
        return {"kind": "sharded", "rank": self.rank, "world": self.world,
                "master": self.master.detach().cpu()}

    def load_state_dict(self, sd: dict):
        """Restore this rank's master shard, then re-sync the live parameters
        from the restored shards (a forced pull)."""
        if sd.get("kind") != "sharded":
            return
        if sd["world"] != self.world or sd["rank"] != self.rank:
            raise ValueError(f"sharded PS checkpoint is for rank {sd['rank']}/{sd['world']}, "
                             f"this is rank {self.rank}/{self.world}")
        with torch.no_grad():
            self.master.copy_(sd["master"].to(self.master.device))
            if self.world > 1 or self.force:
                if dist.get_backend(self.group) == "gloo":
                    self._gloo_all_gather(self.arena.p32).wait()
                else:
                    dist.all_gather_into_tensor(self.arena.p32, self.master, group=self.group)
            else:
                self.arena.p32.copy_(self.master)
        self.arena.refresh_shadow()
        self.arena.bump()


class _EventSpan:
    """Start/end CUDA events on the current stream; kept (bounded) on the client."""

    KEEP = 64

    def __init__(self, client, kind):
        self.client, self.kind = client, kind

    def __enter__(self):
        self.a = torch.cuda.Event(enable_timing=True)
        self.a.record()
        return self

    def __exit__(self, *exc):
        b = torch.cuda.Event(enable_timing=True)
        b.record()
        spans = self.client.__dict__.setdefault("_spans", {})
        lst = spans.setdefault(self.kind, [])
        lst.append((self.a, b))
        if len(lst) > self.KEEP:
            del lst[0]
        return False


class _NullSpan:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


_NULL_SPAN = _NullSpan()


class _EventWork:
    """Adapter so a CUDA event can sit in the send-work slots."""

    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)

    def is_completed(self):
        return self.ev.query()
