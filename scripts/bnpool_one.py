"""Run the fused stem BN + ReLU + max pool kernels (forward, backward) and, for comparison,
the unfused BN apply + max pool pair, on the ResNet-50 bs128 stem shape (128 x 64 x 112 x 112)
for --iters iterations: a driver for rocprofv3 --pmc passes (scripts/gpu_r4pmc.sh)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_ml_pytorch_amd.ops._ext import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--batch", type=int, default=128)
    a = ap.parse_args()
    CL = torch.channels_last
    N, C, H, W = a.batch, 64, 112, 112
    x = torch.randn(N, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    g = torch.rand(C, device="cuda") + 0.5
    b = torch.randn(C, device="cuda") * 0.2
    fs = torch.zeros(2 * 64 * C + 4, device="cuda")
    bs = torch.zeros_like(fs)
    dg = torch.zeros(C, device="cuda")
    db = torch.zeros(C, device="cuda")
    for _ in range(a.iters):
        y, idx, stats, xm = native().bn_relu_maxpool_fwd(x, fs, False, g, b, None, None, 0.1, 1e-5,
                                                          bs, 3, 2, 1)
        dp = torch.ones_like(y)
        native().maxpool_bn_bwd(x, dp, idx, xm, g, stats, dg, db, bs, fs, 3, 2, 1)
        # unfused reference pair (forward): BN apply (+ReLU) then max pool
        yb, st2, _ = native().bn_fwd_fold(x, fs, False, None, g, b, None, None, 0.1, 1e-5, True,
                                          False, bs)
        native().maxpool_fwd(yb, 3, 2, 1, False, False)
        fs.zero_()
        bs.zero_()
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
