#!/usr/bin/env python
"""Headline benchmark: ResNet-18 Downpour/ASGD training throughput (samples/s, whole node).

BASELINE.json metric: "samples/sec (whole node) ResNet-18 ASGD at 1/2/4/8 MI355X".
Config: ResNet-18 (CIFAR stem, 11,173,962 params, random init), synthetic
CIFAR-10-shaped batches resident in HBM, bf16 compute / fp32 master params,
Downpour SGD with n_push = n_pull = 10 (reference defaults, main.py:146-147).

* N = 1: one worker with an in-process PS on the same GPU (push = PS apply
  kernel, pull = snapshot + land), i.e. every ASGD operation still runs.
* N > 1: every rank is a worker; the PS is sharded across all ranks (each
  owns 1/N of the fp32 master): push = reduce-scatter of the accumulated
  deltas + apply, pull = all-gather, both on a side stream over RCCL/xGMI,
  landed with staleness <= 1 step.  Per-GPU batch is fixed (weak scaling).

Timing: W untimed warmup steps, then exactly K steps bracketed by barrier +
``torch.cuda.synchronize()`` on both sides; the max elapsed over ranks is used.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def _sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


METRIC = "samples/sec (whole node) ResNet-18 ASGD at 1/2/4/8 MI355X; time-to-target-loss"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=512,
                    help="per-GPU batch (sweep: profiles/batch_sweep_r1.txt)")
    ap.add_argument("--mode", default="asgd", choices=["asgd", "sync", "single"])
    ap.add_argument("--ps", default="auto", choices=["auto", "local", "sharded", "central"])
    ap.add_argument("--n-push", type=int, default=10)
    ap.add_argument("--n-pull", type=int, default=10)
    ap.add_argument("--staleness", type=int, default=1)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--momentum", type=float, default=0.0)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--graph", type=int, default=1, help="capture fwd+bwd+update in a hipGraph")
    ap.add_argument("--profile-steps", type=int, default=0,
                    help="extra steps after timing, for rocprofv3 windows")
    ap.add_argument("--ttl-target", type=float, default=0.5,
                    help="after the throughput run: train a FRESH model on learnable synthetic "
                         "data until the mean loss of 10 steps <= target and report the "
                         "wall time (the metric's time-to-target-loss half); 0 skips")
    ap.add_argument("--ttl-max-steps", type=int, default=1500)
    return ap.parse_args()


def time_to_target(a, cfg, info):
    """Wall time for a freshly initialised model (same engine, same config) to
    bring the mean training loss over 10 steps down to ``--ttl-target`` on
    class-template synthetic images (learnable, unlike the noise batches of the
    throughput run).  Includes graph capture and the first (tuning) step."""
    from distributed_ml_pytorch_amd.runtime.dist import barrier
    from distributed_ml_pytorch_amd.runtime.trainer import Worker
    from distributed_ml_pytorch_amd.utils.data import DeviceBatchPool

    torch.manual_seed(1000 + info.rank)
    w = Worker(cfg, info)
    if a.mode != "sync":
        w.enable_graph(bool(a.graph))
    pool = DeviceBatchPool(a.batch, w.input_shape, w.num_classes, w.device, n_batches=32,
                           dtype=w.compute_dtype, seed=100 + info.rank, learnable=True)
    barrier(info)
    _sync()
    t0 = time.perf_counter()
    steps, reached, window = 0, False, []
    while steps < a.ttl_max_steps:
        x, y = pool.next()
        loss, _ = w.train_step(x, y)
        window.append(loss.detach().float())
        steps += 1
        if steps % 10 == 0:
            m = torch.stack(window).mean().reshape(1)
            window.clear()
            if info.is_distributed:
                # every rank must take the same stop decision, or the ranks that keep
                # training would block in a push collective the others never join
                dist.all_reduce(m, op=dist.ReduceOp.SUM)
                m /= info.world_size
            mean = float(m.item())
            if mean <= a.ttl_target:
                reached = True
                break
    _sync()
    t = time.perf_counter() - t0
    w.finish()
    return {"time_to_target_s": round(t, 3), "ttl_target_loss": a.ttl_target,
            "ttl_steps": steps, "ttl_reached": reached,
            "ttl_data": "synthetic class-template images (signal 0.5 + N(0,1) noise), "
                        "32 distinct batches per rank"}


def main():
    a = parse()
    from distributed_ml_pytorch_amd.runtime.dist import init_distributed, barrier, shutdown
    from distributed_ml_pytorch_amd.runtime.trainer import TrainConfig, Worker
    from distributed_ml_pytorch_amd.utils.data import DeviceBatchPool

    info = init_distributed(use_cuda=torch.cuda.is_available())
    world = info.world_size
    ps = a.ps
    if ps == "auto":
        ps = "sharded" if world > 1 else "local"
    cfg = TrainConfig(model=a.model, batch_size=a.batch, lr=a.lr, momentum=a.momentum,
                      n_push=a.n_push, n_pull=a.n_pull, staleness=a.staleness, mode=a.mode,
                      ps=ps, dtype=a.dtype, cuda=True, evaluate=False, verbose=False)
    w = Worker(cfg, info)
    graphed = w.enable_graph(bool(a.graph)) if a.mode != "sync" else False
    pool = DeviceBatchPool(a.batch, w.input_shape, w.num_classes, w.device, n_batches=4,
                           dtype=w.compute_dtype, seed=info.rank)
    for _ in range(a.warmup):
        x, y = pool.next()
        loss, _ = w.train_step(x, y)
    barrier(info)
    _sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        x, y = pool.next()
        loss, _ = w.train_step(x, y)
    _sync()
    barrier(info)
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], device=w.device, dtype=torch.float64)
    if info.is_distributed:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    final_loss = float(loss.float().item())
    for _ in range(a.profile_steps):
        x, y = pool.next()
        w.train_step(x, y)
    _sync()
    in_shape = tuple(w.input_shape)
    w.finish()
    ttl = time_to_target(a, cfg, info) if a.ttl_target > 0 else None
    if info.rank == 0:
        global_batch = a.batch * world
        value = global_batch * a.steps / elapsed
        par = {"asgd": f"asgd-{ps}-ps x{world}", "sync": f"dp{world}",
               "single": "single"}[a.mode]
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1e3 * elapsed / a.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": a.dtype,
            "data": f"synthetic ({'x'.join(map(str, in_shape))} images, random labels, "
                    "HBM-resident); random-init weights",
            "config": {"model": (f"{a.model} ({'CIFAR' if in_shape[-1] <= 64 else 'ImageNet'} stem)"
                                 if a.model.startswith("resnet") else a.model),
                       "global_batch": global_batch, "per_gpu_batch": a.batch,
                       "seq_len": None, "image": "x".join(map(str, in_shape)),
                       "parallelism": par, "n_push": a.n_push, "n_pull": a.n_pull,
                       "staleness": a.staleness, "lr": a.lr, "hip_graph": bool(graphed),
                       "master_dtype": "fp32"},
            "final_loss": round(final_loss, 4),
        }
        if ttl is not None:
            out.update(ttl)
        print(json.dumps(out), flush=True)
    shutdown()


if __name__ == "__main__":
    main()
