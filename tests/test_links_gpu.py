"""Link-concurrent central PS (parallel/links.py) on one GPU.

RCCL refuses two ranks on one device, so the per-pair RCCL communicators are
replaced by a transport with the same stream semantics as torch's
ProcessGroupNCCL point-to-point ops: every peer has its own "comm" stream, an
operation makes it wait on the caller's current stream, a ``torch.cuda._sleep``
stands in for the wire time, a device copy moves the bytes, and ``work.wait()``
makes the caller's current stream wait for the copy.  With that, the PS must
(a) have two workers' receives in flight at once, (b) apply each delta only
after its own receive, serially, all of them, and (c) send replies that
observe every apply enqueued before them.
"""
import os
import socket
from collections import defaultdict, deque

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


class _EvWork:
    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)

    def is_completed(self):
        return self.ev.query()


class DelayedCopyTransport:
    def __init__(self, cycles: int):
        self.cycles = cycles
        self.outbox = defaultdict(deque)    # peer -> tensors the peer "sends" to us
        self.inbox = defaultdict(list)      # peer -> tensors we sent to the peer
        self.comm = {}
        self.spans = []

    def _op(self, peer, kind, fn):
        cs = self.comm.get(peer)
        if cs is None:
            cs = self.comm[peer] = torch.cuda.Stream()
        cs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cs):
            a = torch.cuda.Event(enable_timing=True)
            a.record()
            torch.cuda._sleep(self.cycles)
            fn()
            b = torch.cuda.Event(enable_timing=True)
            b.record()
        self.spans.append((kind, peer, a, b))
        return _EvWork(b)

    def irecv(self, buf, peer):
        src = self.outbox[peer].popleft()
        return self._op(peer, "recv", lambda: buf.copy_(src))

    def isend(self, buf, peer):
        out = torch.empty_like(buf)
        self.inbox[peer].append(out)
        return self._op(peer, "send", lambda: out.copy_(buf))


def _gloo_world1():
    if dist.is_initialized():
        return False
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    return True


def test_ps_links_overlap_receives():
    from distributed_ml_pytorch_amd.parallel import messaging as M
    from distributed_ml_pytorch_amd.parallel.server import ParameterServer

    made = _gloo_world1()
    try:
        n = 1 << 20
        tr = DelayedCopyTransport(cycles=20_000_000)
        g = torch.Generator(device="cuda").manual_seed(0)
        deltas = {w: [torch.randn(n, device="cuda", generator=g) for _ in range(2)]
                  for w in (1, 2)}
        for w in (1, 2):
            tr.outbox[w].extend(deltas[w])
        ps = ParameterServer(numel=n, workers=[1, 2], payload="rccl", device="cuda:0",
                             transport=tr, trace_links=True)
        torch.cuda.synchronize()
        GU, PR = M.MessageCode.GradientUpdate, M.MessageCode.ParameterRequest
        f32 = torch.float32
        # two pushes per worker, interleaved as headers would arrive, then a pull
        ps.handle(GU, 1, 0, 0, n, f32)
        ps.handle(GU, 2, 0, 0, n, f32)
        ps.handle(GU, 1, 1, 1, n, f32)
        ps.handle(GU, 2, 1, 1, n, f32)
        ps.handle(PR, 1, 2, 0, 0, f32)
        ps.finish()
        torch.cuda.synchronize()

        # (b) every delta applied exactly once
        want = sum(deltas[1]) + sum(deltas[2])
        torch.testing.assert_close(ps.parameters(), want, rtol=1e-5, atol=1e-5)
        assert ps.version == 4
        # (c) the reply observed all four applies, version trailing
        reply = tr.inbox[1][-1]
        torch.testing.assert_close(reply[:n], want, rtol=1e-5, atol=1e-5)
        assert float(reply[n]) == 4.0

        # (a) receives from different workers overlap in time: worker 2's first
        # receive starts before worker 1's first receive has finished
        recvs = [(p, a, b) for k, p, a, b in tr.spans if k == "recv"]
        (p1, a1, b1), (p2, a2, b2) = recvs[0], recvs[1]
        assert (p1, p2) == (1, 2)
        dur1 = a1.elapsed_time(b1)
        start2 = a1.elapsed_time(a2)
        assert start2 < 0.5 * dur1, (start2, dur1)
        # all four receives took (about) the time of two back-to-back ones per link,
        # not four in series
        t_all = min(a.elapsed_time(b) for _, _, a, b in recvs[:1]) or dur1
        end_last = max(a1.elapsed_time(b) for _, _, _, b in recvs)
        assert end_last < 3.2 * t_all, (end_last, t_all)
        # the same peer's transfers stay ordered on its link: worker 1's second
        # receive starts after its first ended
        w1 = [(a, b) for p, a, b in recvs if p == 1]
        assert a1.elapsed_time(w1[1][0]) >= a1.elapsed_time(w1[0][1]) - 1e-3
        # ring slots: two per (peer, shape), so nothing was reused yet
        assert ps.links.counts["recv"] == 4 and ps.links.counts["send"] == 1
    finally:
        if made:
            dist.destroy_process_group()
