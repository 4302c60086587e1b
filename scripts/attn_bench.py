"""Time the native fused attention (csrc/attention.hip) on the ViT-B/16 shape
(B=64, N=197, H=12, head dim 64): forward and backward, us per call."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from distributed_ml_pytorch_amd.ops._ext import native


def t_us(fn, it=20, rounds=3):
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


B, N, H = 64, 197, 12
D = H * 64
qkv = (torch.randn(B, N, 3 * D, device="cuda") * 0.5).to(torch.bfloat16)
out, lse = native().attention_fwd(qkv, H)
dout = torch.randn_like(out)
f = t_us(lambda: native().attention_fwd(qkv, H))
b = t_us(lambda: native().attention_bwd(qkv, out, dout, lse, H))
flop = 4.0 * B * H * N * N * 64
print(f"fwd {f:.1f} us ({flop / f / 1e6:.0f} TF/s)  "
      f"bwd {b:.1f} us ({2.5 * flop / b / 1e6:.0f} TF/s)", flush=True)
