"""Time every native wgrad tile config on the ViT-B/16 linear weight-gradient
shapes (M = 64 x 197 tokens); prints the best config per tile family."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from distributed_ml_pytorch_amd.ops._ext import native
from distributed_ml_pytorch_amd.ops.conv import _wgrad_candidates


def t_us(fn, it=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / it


M = 64 * 197
for N, K in ((3072, 768), (768, 3072), (2304, 768), (768, 768)):
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    x4 = x.view(M, 1, 1, K).permute(0, 3, 1, 2)
    dy4 = dy.view(M, 1, 1, N).permute(0, 3, 1, 2)
    g = torch.zeros(N, K, 1, 1, device="cuda")
    best = {}
    for c in _wgrad_candidates(K, N):
        fam = 256 if c & 512 else (128 if c & 256 else 64)
        us = t_us(lambda: native().conv_wgrad(dy4, x4, g, 1, 0, c))
        if fam not in best or us < best[fam][0]:
            best[fam] = (us, c)
    tf = 2 * M * N * K / 1e12
    print(f"N={N} K={K}: " + "  ".join(
        f"BMW{f}: {u:.1f} us ({tf / u * 1e6:.0f} TF/s, cfg {c})" for f, (u, c) in sorted(best.items())),
        flush=True)
