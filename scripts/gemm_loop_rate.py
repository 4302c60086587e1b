"""Main-loop rate of the native GEMM tiles per pass (csrc/gemm.hip), separated from the
per-launch costs: one full round of 256 x 256 output tiles (M = N = 4096 -> 256 tiles,
one per CU) timed at growing reduction length K; time = a + b K, loop TF/s = 2 M N / b.
fwd: A [M, K], B [N, K] (both k-contiguous, ds_read_b128 fragments); dgrad: B [K, N]
(k-strided: transposed ds_read_b64_tr_b16 fragments); wgrad: A [K, M], B [K, N] (both
k-strided, fp32 accumulate).  hipBLASLt on the same operands for reference.
Usage: python scripts/gemm_loop_rate.py [--cfgs 0,1,2,4,10] [--mn 4096]"""
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


def fit(ks, ts, M, N):
    xs = torch.tensor([float(k) for k in ks], dtype=torch.float64)
    ys = torch.tensor(ts, dtype=torch.float64)
    A = torch.stack([torch.ones_like(xs), xs], 1)
    sol = torch.linalg.lstsq(A, ys.unsqueeze(1)).solution.squeeze(1)
    return float(sol[0]), 2.0 * M * N / float(sol[1]) / 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="0,1,2,4,10,11")
    ap.add_argument("--mn", type=int, default=4096)
    ap.add_argument("--ks", default="1024,2048,4096")
    a = ap.parse_args()
    M = N = a.mn
    ks = [int(k) for k in a.ks.split(",")]
    cfgs = [int(c) for c in a.cfgs.split(",")]
    r = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).to(torch.bfloat16)  # noqa: E731
    print(f"M = N = {M}: a [us] / main-loop TF/s per pass (fit over K = {ks})")
    for mode, name in ((0, "fwd"), (1, "dgrad"), (2, "wgrad")):
        rows = {}
        for K in ks:
            if mode == 0:
                x, w = r(M, K), r(N, K)
                c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
                blas = lambda: torch.mm(x, w.t(), out=c)  # noqa: E731
                nat = lambda cf: native().gemm(0, 0, cf, x, w, c)  # noqa: E731
            elif mode == 1:
                x, w = r(M, K), r(K, N)
                c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
                blas = lambda: torch.mm(x, w, out=c)  # noqa: E731
                nat = lambda cf: native().gemm(1, 0, cf, x, w, c)  # noqa: E731
            else:
                x, w = r(K, M), r(K, N)
                c = torch.zeros(M, N, device="cuda")
                blas = lambda: torch.ops.aten.addmm.dtype_out(c, x.t(), w, torch.float32, out=c)  # noqa: E731
                nat = lambda cf: native().gemm(2, 3, cf, x, w, c, splits=1)  # noqa: E731
            rows.setdefault("blas", []).append(timeit(blas))
            for cf in cfgs:
                if native().gemm_config_ok(mode, cf):
                    rows.setdefault(cf, []).append(timeit(lambda: nat(cf)))
        line = []
        for k, ts in rows.items():
            aa, tf = fit(ks, ts, M, N)
            line.append(f"{'c' + str(k) if k != 'blas' else 'blas'}: a={aa:5.1f} loop={tf:5.0f} "
                        f"(K={ks[-1]}: {ts[-1]:6.1f} us)")
        print(f"{name:>6}  " + " | ".join(line), flush=True)


if __name__ == "__main__":
    main()
