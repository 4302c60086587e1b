#!/usr/bin/env python
"""Ablation of the native conv tiles on one shape: every config, fwd with/without the
fused BN-stats epilogue, dgrad, and wgrad variants (median ms + TFLOP/s)."""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CL = torch.channels_last


def t(fn, iters=15):
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
    ap.add_argument("--shape", default="256,64,32,32,64,3,1,1")
    ap.add_argument("--repeat", type=int, default=1, help="launches per timed region")
    ap.add_argument("--wgrad-only", action="store_true")
    ap.add_argument("--no-wgrad", action="store_true")
    a = ap.parse_args()
    B, CI, H, W, CO, k, st, pd = map(int, a.shape.split(","))
    from distributed_ml_pytorch_amd.ops._ext import native

    nat = native()
    x = torch.randn(B, CI, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(CO, CI, k, k, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=CL)
    OH = (H + 2 * pd - k) // st + 1
    dy = torch.randn(B, CO, OH, OH, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    dw = torch.zeros(CO, CI, k, k, device="cuda").contiguous(memory_format=CL)
    fl = 2.0 * B * OH * OH * CO * CI * k * k
    print(f"shape {a.shape}  GFLOP {fl / 1e9:.2f}")
    for c in ([] if a.wgrad_only else nat.conv_configs()):
        cid = c[0]
        f1 = t(lambda: nat.conv_fwd(x, w, st, pd, True, cid))
        f0 = t(lambda: nat.conv_fwd(x, w, st, pd, False, cid))
        d = t(lambda: nat.conv_dgrad(dy, w, H, W, st, pd, cid))
        print(f"cfg {cid:2d} {tuple(c[1:])}: fwd+stats {f1:.4f} ({fl / f1 / 1e9:6.1f} TF)  fwd {f0:.4f} "
              f"({fl / f0 / 1e9:6.1f})  dgrad {d:.4f} ({fl / d / 1e9:6.1f})")
    from distributed_ml_pytorch_amd.ops.conv import _wgrad_candidates

    for cfg in ([] if a.no_wgrad else _wgrad_candidates(CI * k * k)):
        ww = t(lambda: nat.conv_wgrad(dy, x, dw, st, pd, cfg))
        print(f"wgrad bnw={64 * (cfg & 3)} bp={32 if cfg & 4 else 64} ns={3 if cfg & 8 else 2} "
              f"chunk={512 * (cfg >> 4)}: {ww:.4f} ({fl / ww / 1e9:6.1f} TF)")


if __name__ == "__main__":
    main()
