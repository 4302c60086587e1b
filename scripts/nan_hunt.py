"""Per-step loss / parameter-norm trace of the bench configuration (ResNet-18 bs512,
ASGD local PS) under graph / eager and asgd / sync: finds the first step at which a
run goes non-finite.  Run on the GPU box."""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
os.environ.setdefault("DMP_CONV_TUNE_SEED", os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "..", "tuning", "mi355x_tune_cache.json"))
import torch

from distributed_ml_pytorch_amd.runtime.dist import DistInfo
from distributed_ml_pytorch_amd.runtime.trainer import TrainConfig, Worker
from distributed_ml_pytorch_amd.utils.data import DeviceBatchPool


def run(mode, graph, steps, model, batch, n_push, learnable):
    torch.manual_seed(0)
    if os.environ.get("NAN_SETDEV") == "1":
        torch.cuda.set_device(0)
    info = DistInfo(device=torch.device("cuda", 0))
    n_pull = int(os.environ.get("NAN_NPULL", n_push))
    extra = dict(dtype="bf16", bucket_mb=32.0, delta_scale="sum", payload="auto",
                 wire_dtype="fp32", momentum=0.0) if os.environ.get("NAN_BENCHCFG") == "1" else {}
    cfg = TrainConfig(model=model, batch_size=batch, lr=0.05, mode=mode, ps="local",
                      n_push=n_push, n_pull=n_pull, staleness=1, cuda=True, evaluate=False,
                      verbose=False, **extra)
    w = Worker(cfg, info)
    w.enable_graph(graph)
    pool = DeviceBatchPool(batch, w.input_shape, w.num_classes, w.device, n_batches=4,
                           dtype=w.compute_dtype, seed=0, learnable=learnable, signal=0.05)
    first_bad = None
    if os.environ.get("NAN_BENCHLIKE") == "1":
        for i in range(10):
            x, y = pool.next()
            loss, _ = w.train_step(x, y)
        torch.cuda.synchronize()
        seen = []
        for i in range(30):
            x, y = pool.next()
            loss, _ = w.train_step(x, y)
            seen.append(loss)
        torch.cuda.synchronize()
        print("  benchlike losses " + " ".join(f"{float(v.float()):.3g}" for v in seen), flush=True)
        print(f"  benchlike: loss after 40 unsynced steps {float(loss.float().item()):.4f} "
              f"|p| {w.param_norm():.4f}", flush=True)
    for i in range(steps):
        x, y = pool.next()
        loss, _ = w.train_step(x, y)
        lv = float(loss.float().item())
        pn = w.param_norm()
        gn = float(w.arena.g32.float().norm()) if w.arena.g32 is not None else float("nan")
        if i < 25 or i % 10 == 0 or not math.isfinite(lv) or not math.isfinite(pn):
            print(f"  {mode:5s} graph={int(graph)} step {i:4d} loss {lv:.4f} |p| {pn:.4f} |g| {gn:.4f}",
                  flush=True)
        if first_bad is None and not (math.isfinite(lv) and math.isfinite(pn)):
            first_bad = i
            break
    w.finish()
    print(f"== {model} {mode} graph={graph} n_push={n_push}: first non-finite step {first_bad}",
          flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--variants", default="asgd:1,asgd:0,sync:1")
    ap.add_argument("--n-push", type=int, default=10)
    ap.add_argument("--learnable", type=int, default=0)
    a = ap.parse_args()
    for v in a.variants.split(","):
        mode, g = v.split(":")
        run(mode, bool(int(g)), a.steps, a.model, a.batch, a.n_push, bool(a.learnable))


if __name__ == "__main__":
    main()
