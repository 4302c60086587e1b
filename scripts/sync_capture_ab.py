"""Price eager vs hipGraph-captured sync DP with REAL RCCL bucket all-reduces on 1 GPU.

A world-size-1 RCCL group with ``force_collectives``: every bucket's all-reduce is
an actual RCCL launch from the grad-ready hooks, exactly as at N > 1, so the
difference between the arms is the host-launch cost of ~350 dispatches per
ResNet-50 step (eager) vs one graph replay (captured).  Interleaved rounds in
one process (cdna_hip_programming.md §5.4 rule 24).

    python scripts/sync_capture_ab.py --model resnet50 --batch 128
"""
import argparse
import os
import socket
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
os.environ.setdefault("DMP_CONV_TUNE_SEED", os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "..", "tuning", "mi355x_tune_cache.json"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    a = ap.parse_args()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)

    from distributed_ml_pytorch_amd.runtime.dist import DistInfo
    from distributed_ml_pytorch_amd.runtime.trainer import TrainConfig, Worker
    from distributed_ml_pytorch_amd.utils.data import DeviceBatchPool

    info = DistInfo(0, 1, 0, "nccl", torch.device("cuda", 0))
    cfg = TrainConfig(model=a.model, batch_size=a.batch, mode="sync", ps="local", lr=0.01,
                      evaluate=False, verbose=False, bucket_mb=a.bucket_mb)
    arms = {}
    for arm in ("eager", "graph"):
        torch.manual_seed(0)
        w = Worker(cfg, info)
        w.ddp.force = True               # real RCCL all-reduces at world 1
        w.use_graph = arm == "graph"
        w.graph = None
        pool = DeviceBatchPool(a.batch, w.input_shape, w.num_classes, w.device, n_batches=4,
                               dtype=w.compute_dtype, seed=1)
        for _ in range(5):
            w.train_step(*pool.next())
        torch.cuda.synchronize()
        arms[arm] = (w, pool)
    times = {k: [] for k in arms}
    for _ in range(a.rounds):
        for arm, (w, pool) in arms.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                loss, _ = w.train_step(*pool.next(), keep=False)
            torch.cuda.synchronize()
            times[arm].append(1e3 * (time.perf_counter() - t0) / a.steps)
            print(f"{arm:6s} {times[arm][-1]:.3f} ms/step loss {float(loss.float()):.4f} "
                  f"graph={w.graph is not None} buckets={w.ddp.num_buckets}", flush=True)
    for arm, ts in times.items():
        print(f"SUMMARY {a.model} bs{a.batch} sync-DP RCCL world1 {arm}: "
              f"median {sorted(ts)[len(ts) // 2]:.3f} min {min(ts):.3f} ms/step", flush=True)
    for w, _ in arms.values():
        w.finish()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
