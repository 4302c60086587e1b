"""Aggregate throughput of K virtual ASGD workers (one HIP stream each) sharing one
parameter server on ONE MI355X (distributed_ml_pytorch_amd/runtime/virtual.py).

    python scripts/virtual_bench.py --k 1 2 4 --model resnet18 --batch 256
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_ml_pytorch_amd.runtime.trainer import TrainConfig  # noqa: E402
from distributed_ml_pytorch_amd.runtime.virtual import VirtualWorkers  # noqa: E402
from distributed_ml_pytorch_amd.utils.data import DeviceBatchPool  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--graph", type=int, default=1)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for k in a.k:
        cfg = TrainConfig(model=a.model, batch_size=a.batch, mode="asgd", lr=0.01, n_push=10,
                          n_pull=10, evaluate=False, verbose=False)
        vw = VirtualWorkers(cfg, k, device=dev)
        vw.enable_graph(bool(a.graph))
        w0 = vw.workers[0]
        pools = [DeviceBatchPool(a.batch, w0.input_shape, w0.num_classes, dev, n_batches=2,
                                 dtype=w0.compute_dtype, seed=i) for i in range(k)]
        for _ in range(a.warmup):
            vw.step([p.next() for p in pools])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            losses = vw.step([p.next() for p in pools])
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        vw.finish()
        torch.cuda.synchronize()
        print(json.dumps({"model": a.model, "virtual_workers": k, "per_worker_batch": a.batch,
                          "steps": a.steps, "hip_graph": bool(a.graph),
                          "ms_per_round": round(1e3 * el / a.steps, 3),
                          "samples_per_s": round(k * a.batch * a.steps / el, 1),
                          "loss": [round(float(l.float()), 3) for l in losses]}), flush=True)
        del vw, pools
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
