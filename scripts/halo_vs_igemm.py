#!/usr/bin/env python
"""ResNet-18 (CIFAR, bs256) 3x3 stride-1 convs: best implicit-GEMM tile vs best
halo-tile config (csrc/conv.hip), forward (+BN partials) and data gradient.

Run on the GPU box with ``PYTHONPATH=$PWD``.
"""
import torch

from distributed_ml_pytorch_amd.ops._ext import native
from distributed_ml_pytorch_amd.ops.conv import _configs

CL = torch.channels_last


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
    print(f"{'shape':>26} {'pass':>6} {'igemm_us':>9} {'cfg':>4} {'halo_us':>8} {'cfg':>4} {'TF igemm/halo':>14}")
    tot_i = tot_h = 0.0
    for B, C, H, W in [(256, 64, 32, 32), (256, 128, 16, 16), (256, 256, 8, 8), (256, 512, 4, 4)]:
        x = torch.randn(B, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        w = (torch.randn(C, C, 3, 3, device="cuda") * 0.02).to(torch.bfloat16).contiguous(memory_format=CL)
        dy = torch.randn(B, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        flop = 2.0 * B * H * W * C * C * 9
        ig = [c[0] for c in _configs() if c[2] <= max(64, C)]
        hc = list(nat.conv_halo_configs(H, W, C, 3, 3, 1, 1))
        for name, run in (("fwd", lambda c: nat.conv_fwd(x, w, 1, 1, True, c)),
                          ("dgrad", lambda c: nat.conv_dgrad(dy, w, H, W, 1, 1, c))):
            ti, ci = min((timeit(lambda c=c: run(c)), c) for c in ig)
            th, ch = min((timeit(lambda c=c: run(c)), c) for c in hc) if hc else (float("nan"), -1)
            tot_i += ti
            tot_h += min(th, ti)
            print(f"{str((B, C, H, W)):>26} {name:>6} {ti:9.1f} {ci:4d} {th:8.1f} {ch:4d} "
                  f"{flop / ti / 1e6:6.0f}/{flop / th / 1e6:.0f}")
        from distributed_ml_pytorch_amd.ops.conv import _wgrad_candidates

        dw = torch.zeros(C, C, 3, 3, device="cuda").contiguous(memory_format=CL)
        run = lambda c: nat.conv_wgrad(dy, x, dw, 1, 1, c)     # noqa: E731
        ti, ci = min((timeit(lambda c=c: run(c)), c) for c in _wgrad_candidates(9 * C))
        hw = list(nat.conv_wgrad_halo_configs(B, H, W, C, C, 3, 3, 1, 1))
        th, ch = min((timeit(lambda c=c: run(c)), c) for c in hw) if hw else (float("nan"), -1)
        tot_i += ti
        tot_h += min(th, ti)
        print(f"{str((B, C, H, W)):>26} {'wgrad':>6} {ti:9.1f} {ci:4d} {th:8.1f} {ch:4d} "
              f"{flop / ti / 1e6:6.0f}/{flop / th / 1e6:.0f}")
    print(f"total igemm {tot_i:.1f} us, with halo where faster {tot_h:.1f} us")


if __name__ == "__main__":
    main()
