#!/usr/bin/env python
"""Does the sharded-PS client's side-stream RCCL traffic overlap the compute
graph replay, at 4 / 8 / 16 hardware queues per process?  

One GPU, a world-1 RCCL group, ``ShardedPSClient(force_collectives=True)``: the
reduce-scatter (push) and all-gather (pull) of the full ResNet-18 arena run on
the client's side stream every ``--every`` steps, exactly as at N > 1, while
the captured fwd+bwd+update graph replays on the compute stream.  Compared
against the same engine with the in-process PS (no collectives): if the side
stream overlaps, the step time barely moves; if its work queues behind the
replay, every comm step pays the collectives' device time.

Each queue count runs in a fresh child process (HIP reads GPU_MAX_HW_QUEUES
once, at initialisation).  Usage: python scripts/hw_queue_overlap.py
"""
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(kind: str, steps: int, every: int, batch: int):
    import torch
    import torch.distributed as dist

    from distributed_ml_pytorch_amd.parallel.clients import LocalPSClient, ShardedPSClient
    from distributed_ml_pytorch_amd.runtime.dist import DistInfo
    from distributed_ml_pytorch_amd.runtime.trainer import TrainConfig, Worker
    from distributed_ml_pytorch_amd.utils.data import DeviceBatchPool

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    info = DistInfo(device=torch.device("cuda", 0))
    cfg = TrainConfig(model="resnet18", batch_size=batch, mode="asgd", ps="local", n_push=every,
                      n_pull=every, lr=0.05, evaluate=False, verbose=False)
    client = ShardedPSClient(staleness=1, force_collectives=True) if kind == "sharded" else \
        LocalPSClient(staleness=1)
    w = Worker(cfg, info, client=client)
    w.enable_graph(True)
    pool = DeviceBatchPool(batch, w.input_shape, w.num_classes, w.device, n_batches=4,
                           dtype=w.compute_dtype, seed=0)
    for _ in range(12):
        x, y = pool.next()
        w.train_step(x, y, keep=False)
    torch.cuda.synchronize()
    best = None
    for _ in range(3):
        t0 = time.perf_counter()
        for _ in range(steps):
            x, y = pool.next()
            w.train_step(x, y, keep=False)
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t0) / steps
        best = ms if best is None else min(best, ms)
    st = w.opt.client.stats() if hasattr(w.opt, "client") else {}
    w.finish()
    dist.destroy_process_group()
    print(json.dumps({"kind": kind, "ms_per_step": round(best, 4),
                      "device_ms": {k: v for k, v in st.items() if "device_ms" in k}}), flush=True)


def main():
    steps, every, batch = 40, 1, 512
    rows = []
    for q in (4, 8, 16):
        for kind in ("local", "sharded"):
            env = dict(os.environ, GPU_MAX_HW_QUEUES=str(q))
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", kind,
                                str(steps), str(every), str(batch)], env=env, cwd=ROOT,
                               capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                print(r.stderr[-3000:], file=sys.stderr)
                sys.exit(r.returncode)
            d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
            d["queues"] = q
            rows.append(d)
            print(json.dumps(d), flush=True)
    print(f"\nResNet-18 bs{batch}, push + pull of the whole arena every {every} step(s), "
          f"world-1 RCCL, best of 3 x {steps} steps")
    print(f"{'queues':>6} {'local ms':>9} {'sharded ms':>11} {'delta ms':>9} "
          f"{'push dev ms':>11} {'pull dev ms':>11} {'hidden %':>8}")
    for q in (4, 8, 16):
        lo = next(r for r in rows if r["queues"] == q and r["kind"] == "local")
        sh = next(r for r in rows if r["queues"] == q and r["kind"] == "sharded")
        dev = sh["device_ms"]
        comm = sum(v for k, v in dev.items() if k in ("push_device_ms", "pull_device_ms"))
        delta = sh["ms_per_step"] - lo["ms_per_step"]
        hidden = 100.0 * (1 - delta / comm) if comm > 0 else float("nan")
        print(f"{q:>6} {lo['ms_per_step']:>9.4f} {sh['ms_per_step']:>11.4f} {delta:>9.4f} "
              f"{dev.get('push_device_ms', 0):>11.4f} {dev.get('pull_device_ms', 0):>11.4f} "
              f"{hidden:>8.1f}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]))
    else:
        main()
