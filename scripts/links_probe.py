"""Which part of the PS link scenario serialises two peers' delayed receives?
Runs tests/test_links_gpu.py's scenario in fresh processes with pieces removed.

    python scripts/links_probe.py
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def raw_pattern(torch, tag, streams=None):
    """probe2's pattern (scripts/stream_overlap_probe.py child_ps2) in this process."""
    C = streams or {p: torch.cuda.Stream() for p in (1, 2)}
    for c in C.values():
        with torch.cuda.stream(c):
            torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    t0 = torch.cuda.Event(enable_timing=True)
    t0.record()
    spans = []
    for p in (1, 2):
        C[p].wait_event(t0)
        with torch.cuda.stream(C[p]):
            a = torch.cuda.Event(enable_timing=True)
            a.record()
            torch.cuda._sleep(20_000_000)
            b = torch.cuda.Event(enable_timing=True)
            b.record()
        spans.append((p, a, b))
    torch.cuda.synchronize()
    print(json.dumps({"variant": tag, "spans": [(p, round(t0.elapsed_time(a), 2),
                                                  round(t0.elapsed_time(b), 2))
                                                 for p, a, b in spans]}), flush=True)


def child(variant: str):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch

    import test_links_gpu as T
    from distributed_ml_pytorch_amd.parallel import messaging as M
    from distributed_ml_pytorch_amd.parallel.server import ParameterServer

    if variant == "raw_first":
        raw_pattern(torch, "raw_first")
        return
    if variant.startswith("cold"):
        cold(torch, T, variant)
        return
    T._gloo_world1()
    n = 1 << 20
    tr = T.DelayedCopyTransport(cycles=20_000_000)
    if variant == "nocopy":
        tr.irecv = lambda buf, peer: tr._op(peer, "recv", lambda: None)
    g = torch.Generator(device="cuda").manual_seed(0)
    for w in (1, 2):
        tr.outbox[w].extend([torch.randn(n, device="cuda", generator=g) for _ in range(3)])
    ps = ParameterServer(numel=n, workers=[1, 2], payload="rccl", device="cuda:0",
                         transport=tr, trace_links=(variant != "notrace"))
    if variant == "noapply":
        ps._apply = lambda delta, ready=None, slot=None: ps.links.release(slot, ps.stream)
    import time

    GU = M.MessageCode.GradientUpdate
    # warm-up round (first-call costs), then a timed round
    ps.handle(GU, 1, 0, 0, n, torch.float32)
    ps.handle(GU, 2, 0, 0, n, torch.float32)
    torch.cuda.synchronize()
    tr.spans.clear()
    t0 = torch.cuda.Event(enable_timing=True)
    t0.record()
    host = []
    for w in (1, 2):
        h = time.perf_counter()
        ps.handle(GU, w, 1, 1, n, torch.float32)
        host.append(round(1e3 * (time.perf_counter() - h), 3))
    torch.cuda.synchronize()
    rec = [(p, round(t0.elapsed_time(a), 2), round(t0.elapsed_time(b), 2))
           for k, p, a, b in tr.spans]
    print(json.dumps({"variant": variant, "recv_spans": rec, "host_ms_per_handle": host}),
          flush=True)
    if variant == "full":
        raw_pattern(torch, "raw_after_ps_new_streams")
        raw_pattern(torch, "raw_after_ps_transport_streams", tr.comm)


def cold(torch, T, variant):
    """The test's first round with nothing warmed ('cold'), with only the
    streams warmed by a tiny kernel ('cold_streams': PairLinks' + the transport's),
    or with only the transport's kernels (sleep, copy) launched once ('cold_kernels')."""
    import time

    from distributed_ml_pytorch_amd.parallel import messaging as M
    from distributed_ml_pytorch_amd.parallel.server import ParameterServer

    T._gloo_world1()
    n = 1 << 20
    tr = T.DelayedCopyTransport(cycles=20_000_000)
    for w in (1, 2):
        tr.outbox[w].extend([torch.randn(n, device="cuda") for _ in range(2)])
    ps = ParameterServer(numel=n, workers=[1, 2], payload="rccl", device="cuda:0",
                         transport=tr, trace_links=True)
    if variant == "cold_streams":
        for s_ in list(tr.comm.values()) + list(ps.links._streams.values()):
            with torch.cuda.stream(s_):
                torch.zeros(1, device="cuda")
    if variant == "cold_kernels":
        a = torch.zeros(n, device="cuda")
        torch.cuda._sleep(1000)
        a.copy_(tr.outbox[1][0])
        torch.cuda.Event(enable_timing=True).record()
    torch.cuda.synchronize()
    GU = M.MessageCode.GradientUpdate
    t0 = torch.cuda.Event(enable_timing=True)
    t0.record()
    host = []
    for w in (1, 2):
        h = time.perf_counter()
        ps.handle(GU, w, 0, 0, n, torch.float32)
        host.append(round(1e3 * (time.perf_counter() - h), 3))
    torch.cuda.synchronize()
    rec = [(p, round(t0.elapsed_time(a), 2), round(t0.elapsed_time(b), 2))
           for k, p, a, b in tr.spans]
    print(json.dumps({"variant": variant, "recv_spans": rec, "host_ms_per_handle": host}),
          flush=True)


def main():
    if len(sys.argv) > 1:
        child(sys.argv[1])
        return
    qs = os.environ.get("PROBE_QUEUES", "None,8,16,32").split(",")
    vs = os.environ.get("PROBE_VARIANTS", "raw_first,full").split(",")
    for q in [None if q == "None" else q for q in qs]:
        env = dict(os.environ)
        if q:
            env["GPU_MAX_HW_QUEUES"] = q
        for v in vs:
            r = subprocess.run([sys.executable, os.path.abspath(__file__), v], capture_output=True,
                               text=True, timeout=120, cwd=ROOT, env=env)
            out = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            for ln in out or [f"{v}: rc={r.returncode} {r.stderr[-1500:]}"]:
                print(f"queues={q} {ln}", flush=True)


if __name__ == "__main__":
    main()
