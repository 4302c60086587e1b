"""A/B of the split-major XCD deal of the weight-gradient split-K (csrc/gemm.hip
GemmArgs::xcd_k) on the ViT-B/16 dW shapes, same process, interleaved rounds.
Usage (GPU): python scripts/gemm_xcd_ab.py"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_ml_pytorch_amd.ops._ext import native  # noqa: E402


def timeit(fn, reps=20):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    nat = native()
    T = 64 * 197
    # (out, in, cfg, splits, slab): committed picks first, then alternatives
    rows = [(2304, 768, 4, 4, True), (3072, 768, 4, 3, True), (768, 3072, 4, 3, False),
            (768, 768, 9, 6, False), (2304, 768, 4, 8, True), (2304, 768, 0, 8, True),
            (3072, 768, 4, 6, True), (768, 3072, 4, 6, True), (768, 768, 4, 8, True)]
    print(f"{'dW shape':>12} {'cfg':>3} {'s':>2} {'slab':>5} {'old us':>7} {'new us':>7} {'delta':>7}  TF new  maxdiff")
    for M, N, cfg, s, slab in rows:
        dy = torch.randn(T, M, device="cuda").to(torch.bfloat16)
        x = torch.randn(T, N, device="cuda").to(torch.bfloat16)
        g = torch.zeros(M, N, device="cuda")
        outs = []
        for flag in (0, 1):
            nat.gemm_set_xcd_k(flag)
            gg = torch.zeros(M, N, device="cuda")
            nat.gemm(2, 3, cfg, dy, x, gg, None, None, None, None, s, False, None, slab)
            outs.append(gg)
        diff = float((outs[0] - outs[1]).abs().max() / outs[0].abs().max())
        t = {0: [], 1: []}
        for r in range(7):
            for flag in ((0, 1) if r % 2 == 0 else (1, 0)):
                nat.gemm_set_xcd_k(flag)
                t[flag].append(timeit(lambda: nat.gemm(2, 3, cfg, dy, x, g, None, None, None,
                                                       None, s, False, None, slab)))
        o, n = statistics.median(t[0]), statistics.median(t[1])
        print(f"{M:>5}x{N:<6} {cfg:>3} {s:>2} {str(slab):>5} {o:7.1f} {n:7.1f} {100 * (n / o - 1):+6.1f}%"
              f"  {2.0 * T * M * N / n / 1e6:6.0f}  {diff:.1e}", flush=True)
    nat.gemm_set_xcd_k(1)


if __name__ == "__main__":
    main()
