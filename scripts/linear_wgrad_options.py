#!/usr/bin/env python
"""ViT-B/16 linear weight gradients (dW[out][in] = dY^T X over 64*197 tokens):
native 1x1-conv wgrad kernel (fp32 atomics into the arena) vs hipBLASLt with
bf16 output (+ an fp32 add into the arena) vs hipBLASLt fp32-out addmm.

Run on the GPU box with ``PYTHONPATH=$PWD``; prints per-shape microseconds.
"""
import torch

from distributed_ml_pytorch_amd.ops._ext import native
from distributed_ml_pytorch_amd.ops.conv import _wgrad_candidates


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    nat = native()
    M = 64 * 197
    print(f"{'shape':>14} {'native':>8} {'cfg':>4} {'bf16mm':>8} {'bf16mm+add':>11} {'f32addmm':>9}  TF(native/bf16mm)")
    for K, N in [(768, 2304), (768, 768), (768, 3072), (3072, 768)]:
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        g = torch.zeros(N, K, device="cuda")
        flop = 2.0 * M * N * K
        x4 = x.view(M, 1, 1, K).permute(0, 3, 1, 2)
        dy4 = dy.view(M, 1, 1, N).permute(0, 3, 1, 2)
        g4 = g.view(N, K, 1, 1)
        tn, cfg = min((timeit(lambda c=c: nat.conv_wgrad(dy4, x4, g4, 1, 0, c)), c)
                      for c in _wgrad_candidates(K, N))
        tb = timeit(lambda: torch.mm(dy.t(), x))
        tba = timeit(lambda: g.add_(torch.mm(dy.t(), x)))
        tf = timeit(lambda: torch.ops.aten.addmm.dtype_out(g, dy.t(), x, torch.float32, out=g))
        ref = dy.float().t() @ x.float()
        g.zero_()
        nat.conv_wgrad(dy4, x4, g4, 1, 0, cfg)
        e_nat = ((g - ref).norm() / ref.norm()).item()
        e_b = ((torch.mm(dy.t(), x).float() - ref).norm() / ref.norm()).item()
        print(f"{K:>6}->{N:<6} {tn:8.1f} {cfg:4d} {tb:8.1f} {tba:11.1f} {tf:9.1f}  "
              f"{flop / tn / 1e6:.0f}/{flop / tb / 1e6:.0f}  relerr native {e_nat:.1e} bf16 {e_b:.1e}")


if __name__ == "__main__":
    main()
