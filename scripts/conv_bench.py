#!/usr/bin/env python
"""Per-layer timing: native NHWC implicit-GEMM conv vs MIOpen (F.conv2d) on ResNet-18 shapes.

Times fwd, dgrad and wgrad separately with HIP events (median of N), same bf16
channels_last inputs for both.  Prints a table and TFLOP/s.
"""
import argparse
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CL = torch.channels_last


def resnet18_shapes(B):
    s = []
    for cin, cout, hw, stride in [(64, 64, 32, 1), (64, 128, 32, 2), (128, 128, 16, 1),
                                  (128, 256, 16, 2), (256, 256, 8, 1), (256, 512, 8, 2),
                                  (512, 512, 4, 1)]:
        s.append((B, cin, hw, hw, cout, 3, stride, 1))
        if stride == 2:
            s.append((B, cin, hw, hw, cout, 1, 2, 0))
    return s


def timeit(fn, iters):
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
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from distributed_ml_pytorch_amd.ops._ext import native

    nat = native()
    print(f"{'shape':44s} {'pass':6s} {'native_ms':>10s} {'miopen_ms':>10s} {'native_TF':>9s} {'miopen_TF':>9s}")
    tot_n = tot_m = 0.0
    for (B, CI, H, W, CO, k, st, pd) in resnet18_shapes(a.batch):
        x = torch.randn(B, CI, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        w = (torch.randn(CO, CI, k, k, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=CL)
        OH = (H + 2 * pd - k) // st + 1
        flops = 2.0 * B * OH * OH * CO * CI * k * k
        dy = torch.randn(B, CO, OH, OH, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        dw = torch.zeros(CO, CI, k, k, device="cuda").contiguous(memory_format=CL)
        from distributed_ml_pytorch_amd.ops import conv as C
        cf = C._fwd_cfg(x, w, st, pd)
        cd = C._dgrad_cfg(dy, w, H, W, st, pd)
        cw = C._wgrad_cfg(dy, x, tuple(w.shape), st, pd)
        tn_f = timeit(lambda: nat.conv_fwd(x, w, st, pd, True, cf), a.iters)
        tm_f = timeit(lambda: F.conv2d(x, w, None, st, pd), a.iters)
        tn_d = timeit(lambda: nat.conv_dgrad(dy, w, H, W, st, pd, cd), a.iters)
        tn_w = timeit(lambda: nat.conv_wgrad(dy, x, dw, st, pd, cw), a.iters)

        def mi_bwd(mask):
            return torch.ops.aten.convolution_backward(dy, x, w, None, [st, st], [pd, pd], [1, 1],
                                                       False, [0, 0], 1, mask)
        tm_d = timeit(lambda: mi_bwd([True, False, False]), a.iters)
        tm_w = timeit(lambda: mi_bwd([False, True, False]), a.iters)
        name = f"B{B} {CI}->{CO} {H}x{W} k{k} s{st} [{cf},{cd},{cw}]"
        for p, tn, tm in (("fwd", tn_f, tm_f), ("dgrad", tn_d, tm_d), ("wgrad", tn_w, tm_w)):
            print(f"{name:44s} {p:6s} {tn:10.4f} {tm:10.4f} {flops / tn / 1e9:9.1f} {flops / tm / 1e9:9.1f}")
            tot_n += tn
            tot_m += tm
    print(f"TOTAL native {tot_n:.3f} ms   miopen {tot_m:.3f} ms   ratio {tot_m / tot_n:.2f}x")


if __name__ == "__main__":
    main()
