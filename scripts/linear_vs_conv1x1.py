#!/usr/bin/env python
"""ViT-B/16 linear-layer GEMMs: hipBLASLt (F.linear / fp32-out addmm) vs the
native implicit-GEMM conv kernels run as 1x1 convolutions (fwd / dgrad / wgrad).

Prints per-shape times so the routing decision for ``ops.linear`` is measured.
"""
import torch
import torch.nn.functional as F

from distributed_ml_pytorch_amd.ops._ext import native
from distributed_ml_pytorch_amd.ops.conv import _configs, _wgrad_candidates


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
    return a.elapsed_time(b) / reps


def main():
    nat = native()
    M = 64 * 197
    shapes = [(768, 2304), (768, 768), (768, 3072), (3072, 768)]   # (in, out)
    print(f"{'shape':>16} {'pass':>6} {'blas_us':>9} {'native_us':>10} {'cfg':>5}  TF(blas/native)")
    for K, N in shapes:
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
        dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        g = torch.zeros(N, K, device="cuda")
        flop = 2.0 * M * N * K
        x4 = x.view(M, 1, 1, K).permute(0, 3, 1, 2)          # NCHW view, channels_last memory
        w4 = w.view(N, K, 1, 1).contiguous(memory_format=torch.channels_last)
        dy4 = dy.view(M, 1, 1, N).permute(0, 3, 1, 2)
        g4 = g.view(N, K, 1, 1)
        # forward
        tb = timeit(lambda: F.linear(x, w))
        best = min((timeit(lambda c=c: nat.conv_fwd(x4, w4, 1, 0, False, c)), c)
                   for c, *_ in _configs())
        print(f"{K:>7}->{N:<7} {'fwd':>6} {tb*1e3:9.1f} {best[0]*1e3:10.1f} {best[1]:5d}  "
              f"{flop/tb/1e9:.0f}/{flop/best[0]/1e9:.0f}")
        # data gradient (dx = dy @ w): conv dgrad with W^T
        tb = timeit(lambda: dy @ w)
        wt = w4.permute(1, 0, 2, 3).contiguous(memory_format=torch.channels_last)
        best = min((timeit(lambda c=c: nat.conv_dgrad(dy4, w4, 1, 1, 1, 0, c, wt)), c)
                   for c, *_ in _configs())
        print(f"{K:>7}->{N:<7} {'dgrad':>6} {tb*1e3:9.1f} {best[0]*1e3:10.1f} {best[1]:5d}  "
              f"{flop/tb/1e9:.0f}/{flop/best[0]/1e9:.0f}")
        # weight gradient accumulated in fp32
        tb = timeit(lambda: torch.ops.aten.addmm.dtype_out(g, dy.t(), x, torch.float32, out=g))
        best = min((timeit(lambda c=c: nat.conv_wgrad(dy4, x4, g4, 1, 0, c)), c)
                   for c in _wgrad_candidates(K, N))
        print(f"{K:>7}->{N:<7} {'wgrad':>6} {tb*1e3:9.1f} {best[0]*1e3:10.1f} {best[1]:5d}  "
              f"{flop/tb/1e9:.0f}/{flop/best[0]/1e9:.0f}")


if __name__ == "__main__":
    main()
