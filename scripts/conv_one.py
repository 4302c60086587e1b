#!/usr/bin/env python
"""Run ONE native conv pass/config repeatedly (for rocprofv3 --pmc on a single kernel)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CL = torch.channels_last


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="256,64,32,32,64,3,1,1")
    ap.add_argument("--op", choices=["fwd", "dgrad", "wgrad"], default="fwd")
    ap.add_argument("--cfg", type=int, default=-1)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    B, CI, H, W, CO, k, st, pd = map(int, a.shape.split(","))
    from distributed_ml_pytorch_amd.ops._ext import native

    nat = native()
    x = torch.randn(B, CI, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(CO, CI, k, k, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=CL)
    OH = (H + 2 * pd - k) // st + 1
    dy = torch.randn(B, CO, OH, OH, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    dw = torch.zeros(CO, CI, k, k, device="cuda").contiguous(memory_format=CL)
    for _ in range(a.iters):
        if a.op == "fwd":
            nat.conv_fwd(x, w, st, pd, True, a.cfg)
        elif a.op == "dgrad":
            nat.conv_dgrad(dy, w, H, W, st, pd, a.cfg)
        else:
            nat.conv_wgrad(dy, x, dw, st, pd, a.cfg)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
