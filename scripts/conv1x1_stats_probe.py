"""ResNet-18 stride-2 shortcut 1x1 convs (run at stride 1 on the subsampled input):
forward with / without the fused BN-statistics epilogue, every implicit-GEMM tile and
the GEMM route; us per call (min of 3x10)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from distributed_ml_pytorch_amd.ops._ext import native
from distributed_ml_pytorch_amd.ops.conv import _gemm1x1_fwd, BN_SLOTS

CL = torch.channels_last


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


nat = native()
for B, CI, H, CO in ((512, 64, 16, 128), (512, 128, 8, 256), (512, 256, 4, 512)):
    x = torch.randn(B, CI, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(CO, CI, 1, 1, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=CL)
    mb = (x.numel() + B * CO * H * H) * 2 / 1e6
    st = {c[0]: t_us(lambda c=c: nat.conv_fwd(x, w, 1, 0, True, c[0])) for c in nat.conv_configs()}
    ns = {c[0]: t_us(lambda c=c: nat.conv_fwd(x, w, 1, 0, False, c[0])) for c in nat.conv_configs()}
    part = torch.zeros(2 * BN_SLOTS * CO + 4, device="cuda")
    g = t_us(lambda: _gemm1x1_fwd(x, w, part))
    g0 = t_us(lambda: _gemm1x1_fwd(x, w, None))
    bs, bn = min(st, key=st.get), min(ns, key=ns.get)
    print(f"B{B} {CI}->{CO} {H}x{H} ({mb:.0f} MB): igemm+stats best {bs} {st[bs]:.1f} us | igemm no-stats best "
          f"{bn} {ns[bn]:.1f} us | gemm+stats {g:.1f} no-stats {g0:.1f} | roofline@5.5TB/s {mb / 5.5:.1f} us", flush=True)
