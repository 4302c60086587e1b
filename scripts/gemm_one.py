"""Run ONE GEMM (native cfg or hipBLASLt) repeatedly -- a rocprofv3 --pmc target.
Usage: python scripts/gemm_one.py --pass fwd --K 768 --N 2304 --cfg 0 [--blas] [--reps 20]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_ml_pytorch_amd.ops._ext import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pass", dest="p", default="fwd", choices=["fwd", "dgrad", "wgrad"])
    ap.add_argument("--M", type=int, default=12608)
    ap.add_argument("--K", type=int, default=768)
    ap.add_argument("--N", type=int, default=2304)
    ap.add_argument("--cfg", type=int, default=0)
    ap.add_argument("--splits", type=int, default=1)
    ap.add_argument("--blas", action="store_true")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    M, K, N, dev = a.M, a.K, a.N, "cuda"
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = torch.randn(N, K, device=dev).to(torch.bfloat16)
    dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    g = torch.zeros(N, K, device=dev)
    if a.blas:
        fn = {"fwd": lambda: torch.nn.functional.linear(x, w),
              "dgrad": lambda: dy @ w,
              "wgrad": lambda: torch.ops.aten.addmm.dtype_out(g, dy.t(), x, torch.float32,
                                                              out=g)}[a.p]
    else:
        fn = {"fwd": lambda: native().gemm(0, 0, a.cfg, x, w, y),
              "dgrad": lambda: native().gemm(1, 0, a.cfg, dy, w, dx),
              "wgrad": lambda: native().gemm(2, 3, a.cfg, dy, x, g, splits=a.splits)}[a.p]
    for _ in range(a.reps):
        fn()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
