#!/usr/bin/env python
"""Stem conv (few input channels): native VALU kernels vs MIOpen, fwd (+BN stats) and wgrad."""
import argparse
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CL = torch.channels_last


def t(fn, iters=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="256,3,32,32,64,3,1,1;64,3,224,224,64,7,2,3;128,3,227,227,64,11,4,2")
    a = ap.parse_args()
    from distributed_ml_pytorch_amd.ops._ext import native

    nat = native()
    for sh in a.shapes.split(";"):
        B, CI, H, W, CO, k, st, pd = map(int, sh.split(","))
        x = torch.randn(B, CI, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        w = (torch.randn(CO, CI, k, k, device="cuda") * 0.1).to(torch.bfloat16).contiguous(memory_format=CL)
        OH = (H + 2 * pd - k) // st + 1
        OW = (W + 2 * pd - k) // st + 1
        dy = torch.randn(B, CO, OH, OW, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        dw = torch.zeros(CO, CI, k, k, device="cuda").contiguous(memory_format=CL)
        fl = 2.0 * B * OH * OW * CO * CI * k * k
        f_n = t(lambda: nat.conv_small_fwd(x, w, st, pd, True))
        f_m = t(lambda: F.conv2d(x, w, None, st, pd))
        w_n = t(lambda: nat.conv_small_wgrad(dy, x, dw, st, pd))
        w_m = t(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, (st, st), (pd, pd), (1, 1), False, (0, 0), 1, (False, True, False)))
        print(f"{sh:32s} fwd+stats native {f_n * 1e3:8.1f} us  miopen fwd {f_m * 1e3:8.1f} us | "
              f"wgrad native {w_n * 1e3:8.1f} us  miopen {w_m * 1e3:8.1f} us  ({fl / 1e9:.2f} GFLOP)")


if __name__ == "__main__":
    main()
