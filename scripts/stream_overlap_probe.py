"""Do work items on two (or N) HIP streams overlap on this box?  Each arm runs in
a fresh process (HIP reads GPU_MAX_HW_QUEUES at initialisation).

    python scripts/stream_overlap_probe.py            # parent: runs the arms
"""
import json
import os
import subprocess
import sys


def child(kind: str, nstreams: int):
    import torch

    cycles = 20_000_000
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    # warm
    for s in streams:
        with torch.cuda.stream(s):
            torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    t0 = torch.cuda.Event(enable_timing=True)
    t0.record()
    spans = []
    for s in streams:
        s.wait_event(t0)
        with torch.cuda.stream(s):
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            if kind == "sleep":
                torch.cuda._sleep(cycles)
            else:
                x = torch.empty(1 << 26, device="cuda")
                for _ in range(4):
                    x.mul_(1.0001)
            b.record()
            spans.append((a, b))
    torch.cuda.synchronize()
    starts = [t0.elapsed_time(a) for a, _ in spans]
    ends = [t0.elapsed_time(b) for _, b in spans]
    durs = [a.elapsed_time(b) for a, b in spans]
    print(json.dumps({"kind": kind, "n": nstreams, "queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                      "starts": [round(v, 2) for v in starts], "ends": [round(v, 2) for v in ends],
                      "durs": [round(v, 2) for v in durs], "total": round(max(ends), 2)}),
          flush=True)


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "ps":
        child_ps(int(sys.argv[2]))
        return
    if len(sys.argv) > 2 and sys.argv[1] == "ps2":
        child_ps2(int(sys.argv[2]))
        return
    if len(sys.argv) > 2:
        child(sys.argv[1], int(sys.argv[2]))
        return
    if len(sys.argv) > 1 and sys.argv[1] == "ps-arms":
        main_ps()
        return
    for q in (None, "8"):
        for kind in ("sleep", "mul"):
            for n in (2, 4):
                env = dict(os.environ)
                if q is not None:
                    env["GPU_MAX_HW_QUEUES"] = q
                r = subprocess.run([sys.executable, os.path.abspath(__file__), kind, str(n)],
                                   capture_output=True, text=True, timeout=120, env=env)
                out = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
                print(out[-1] if out else f"rc={r.returncode} {r.stderr[-800:]}", flush=True)



def child_ps(wait_apply: int):
    """The link test's stream pattern: apply stream A, per-peer link streams L1, L2
    and comm streams C1, C2 created in that order; C1, C2 sleep (the wire); A waits
    for L1's ready event (wait_apply=1) before C2's work is enqueued."""
    import torch

    cycles = 20_000_000
    A = torch.cuda.Stream()
    streams = {}
    t0 = torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    t0.record()
    spans = []
    for peer in (1, 2):
        L = torch.cuda.Stream()
        C = torch.cuda.Stream()
        streams[peer] = (L, C)
        L.wait_event(t0)
        C.wait_stream(L)
        with torch.cuda.stream(C):
            a = torch.cuda.Event(enable_timing=True)
            a.record()
            torch.cuda._sleep(cycles)
            b = torch.cuda.Event(enable_timing=True)
            b.record()
        spans.append((a, b))
        L.wait_event(b)
        ready = torch.cuda.Event()
        ready.record(L)
        if wait_apply:
            A.wait_event(ready)
            with torch.cuda.stream(A):
                torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    print(json.dumps({"kind": f"ps_pattern wait_apply={wait_apply}",
                      "queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                      "starts": [round(t0.elapsed_time(a), 2) for a, _ in spans],
                      "ends": [round(t0.elapsed_time(b), 2) for _, b in spans]}), flush=True)


def child_ps2(wait_apply: int):
    """As child_ps with every stream created (and warmed) BEFORE t0, and the host
    time of each wait_event call measured: does hipStreamWaitEvent on a pending
    cross-stream event block the host?"""
    import time

    import torch

    cycles = 20_000_000
    A = torch.cuda.Stream()
    LC = {p: (torch.cuda.Stream(), torch.cuda.Stream()) for p in (1, 2)}
    for s_ in [A] + [s_ for pair in LC.values() for s_ in pair]:
        with torch.cuda.stream(s_):
            torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    t0 = torch.cuda.Event(enable_timing=True)
    t0.record()
    spans, host = [], []
    h_start = time.perf_counter()
    for peer in (1, 2):
        L, C = LC[peer]
        L.wait_event(t0)
        C.wait_stream(L)
        with torch.cuda.stream(C):
            a = torch.cuda.Event(enable_timing=True)
            a.record()
            torch.cuda._sleep(cycles)
            b = torch.cuda.Event(enable_timing=True)
            b.record()
        spans.append((a, b))
        h = time.perf_counter()
        L.wait_event(b)
        host.append(round(1e3 * (time.perf_counter() - h), 3))
        ready = torch.cuda.Event()
        ready.record(L)
        if wait_apply:
            h = time.perf_counter()
            A.wait_event(ready)
            host.append(round(1e3 * (time.perf_counter() - h), 3))
            with torch.cuda.stream(A):
                torch.cuda._sleep(1000)
    h_total = round(1e3 * (time.perf_counter() - h_start), 3)
    torch.cuda.synchronize()
    print(json.dumps({"kind": f"ps_pattern2 wait_apply={wait_apply}",
                      "queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                      "starts": [round(t0.elapsed_time(a), 2) for a, _ in spans],
                      "ends": [round(t0.elapsed_time(b), 2) for _, b in spans],
                      "host_wait_ms": host, "host_enqueue_ms": h_total}), flush=True)


def main_ps():
    for q in (None, "16"):
        for wa in (0, 1):
            env = dict(os.environ)
            if q is not None:
                env["GPU_MAX_HW_QUEUES"] = q
            for kind in ("ps", "ps2"):
                r = subprocess.run([sys.executable, os.path.abspath(__file__), kind, str(wa)],
                                   capture_output=True, text=True, timeout=120, env=env)
                out = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
                print(out[-1] if out else f"rc={r.returncode} {r.stderr[-800:]}", flush=True)


if __name__ == "__main__":
    main()
