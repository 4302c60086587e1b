#!/usr/bin/env python
"""Inference-forward driver for rocprofv3: the reference's evaluation loop
(/root/reference/example/main.py:110-125: the whole test set in one batch of
10000 under no_grad) on a model of the registry, bf16, arena-backed weights.
Prints the forward time and, with --check-kernels FILE (a rocprofv3
kernel_stats.csv from a previous run), nothing else -- the summary is made by
scripts/eval_kernels.py."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("DMP_CONV_TUNE_SEED", os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning", "mi355x_tune_cache.json"))

import torch  # noqa: E402

from distributed_ml_pytorch_amd.models import build_model  # noqa: E402
from distributed_ml_pytorch_amd.ops.eval_fold import fold_session  # noqa: E402
from distributed_ml_pytorch_amd.ops.functional import softmax_cross_entropy  # noqa: E402
from distributed_ml_pytorch_amd.parallel.arena import attach_arena  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="alexnet")
    ap.add_argument("--batch", type=int, default=10000)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    torch.manual_seed(0)
    m, shape, nc = build_model(a.model)
    m = m.cuda().eval()
    attach_arena(m, shadow_dtype=torch.bfloat16, channels_last=True)
    x = torch.randn(a.batch, *shape, device="cuda").to(torch.bfloat16)
    if x.dim() == 4:
        x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, nc, (a.batch,), device="cuda")
    # one fold per evaluation pass, as Worker.evaluate does
    with torch.no_grad(), fold_session():
        for _ in range(2):                     # tuning + warm-up
            softmax_cross_entropy(m(x), y)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            loss, hits = softmax_cross_entropy(m(x), y)
        torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / a.iters
    print(f"{a.model} eval forward bs{a.batch}: {ms:.3f} ms ({a.batch / ms * 1e3:.0f} samples/s), "
          f"loss {float(loss):.4f}", flush=True)


if __name__ == "__main__":
    main()
