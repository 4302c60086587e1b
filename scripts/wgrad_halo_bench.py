"""Time every 3x3 stride-1 halo weight-gradient config (csrc/conv_wgrad.hip) on the
ResNet-18 CIFAR stride-1 layers at the bench batch; prints per (NS, TR) variant the
best time and TF/s, plus the gather-kernel best.  DMP_WGRAD_HALO_DIAG=store swaps the
fp32 atomics for plain stores (wrong result, timing of the reduction traffic only)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from distributed_ml_pytorch_amd.ops._ext import native
from distributed_ml_pytorch_amd.ops.conv import _wgrad_candidates

CL = torch.channels_last
VARIANTS = {0: "NS2 TR1", 1: "NS3 TR1", 2: "NS4 TR1", 3: "NS2 TR3", 4: "NS3 TR3", 5: "NS2 TR1 PG2"}


def t_us(fn, it=10, rounds=3):
    fn()
    best = float("inf")
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(it):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / it)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--gather", type=int, default=1)
    a = ap.parse_args()
    nat = native()
    base = 1000
    for C, HW in ((64, 32), (128, 16), (256, 8), (512, 4)):
        B = a.batch
        x = torch.randn(B, C, HW, HW, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        dy = torch.randn(B, C, HW, HW, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        dw = torch.zeros(C, C, 3, 3, device="cuda").contiguous(memory_format=CL)
        tf = 2.0 * B * HW * HW * C * C * 9 / 1e12
        best = {}
        for c in nat.conv_wgrad_halo_configs(B, HW, HW, C, C, 3, 3, 1, 1):
            us = t_us(lambda: nat.conv_wgrad(dy, x, dw, 1, 1, c))
            v = (c - base) // 12
            if v not in best or us < best[v][0]:
                best[v] = (us, c)
        line = f"C={C:3d} {HW}x{HW} B{B}:"
        for v, (us, c) in sorted(best.items()):
            line += f"  [{VARIANTS[v]}] {us:6.1f} us {tf / us * 1e6:5.0f} TF/s (cfg {c})"
        if a.gather:
            g = min(t_us(lambda: nat.conv_wgrad(dy, x, dw, 1, 1, c)) for c in _wgrad_candidates(9 * C, C))
            line += f"  [gather] {g:6.1f} us"
        print(line, flush=True)


if __name__ == "__main__":
    main()
