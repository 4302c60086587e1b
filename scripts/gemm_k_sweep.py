"""Fixed vs per-k cost of the native GEMM tiles (csrc/gemm.hip) against hipBLASLt:
fwd C[M, N] = X[M, K] W[N, K]^T at growing K for the ViT-B/16 QKV output
(M = 12608 tokens, N = 2304).  time(K) ~ a + b K: b = main-loop cost per k
(-> main-loop TF/s), a = per-launch prologue / epilogue / quantisation cost.
Usage: python scripts/gemm_k_sweep.py [--n 2304] [--cfgs 0,5,6,10,14]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_ml_pytorch_amd.ops._ext import native  # noqa: E402


def timeit(fn, reps=10, rounds=3):
    fn()
    best = float("inf")
    for _ in range(rounds):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(1_000_000)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) / reps * 1e3)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=12608)
    ap.add_argument("--n", type=int, default=2304)
    ap.add_argument("--cfgs", default="0,5,6,10,14")
    ap.add_argument("--ks", default="768,1536,3072,6144")
    a = ap.parse_args()
    cfgs = [int(c) for c in a.cfgs.split(",")]
    ks = [int(k) for k in a.ks.split(",")]
    M, N = a.m, a.n
    print(f"M={M} N={N}: us per call (min of 3 rounds x 10), TF/s in brackets")
    print(f"{'K':>6} {'blas':>14} " + " ".join(f"{'c' + str(c):>14}" for c in cfgs))
    rows = {}
    for K in ks:
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        b = torch.zeros(N, device="cuda", dtype=torch.bfloat16)
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        t = {"blas": timeit(lambda: torch.addmm(b, x, w.t(), out=y))}
        for c in cfgs:
            t[c] = timeit(lambda: native().gemm(0, 0, c, x, w, y, bias=b))
        rows[K] = t
        print(f"{K:>6} " + " ".join(f"{t[k]:7.1f} ({fl / t[k] / 1e6:4.0f})"
                                    for k in ["blas"] + cfgs), flush=True)
    # least-squares a + b K per kernel
    print("fit time = a + b*K:  a [us]   main-loop TF/s (= 2MN / b)")
    for k in ["blas"] + cfgs:
        xs = torch.tensor([float(K) for K in ks], dtype=torch.float64)
        ys = torch.tensor([rows[K][k] for K in ks], dtype=torch.float64)
        A = torch.stack([torch.ones_like(xs), xs], 1)
        sol = torch.linalg.lstsq(A, ys.unsqueeze(1)).solution.squeeze(1)
        print(f"{str(k):>6}  a={float(sol[0]):7.1f}  loop={2.0 * M * N / float(sol[1]) / 1e6:6.0f}")


if __name__ == "__main__":
    main()
