"""Native MFMA GEMM (csrc/gemm.hip) vs hipBLASLt (torch.matmul) on the ViT-B/16
linear shapes (bs64: M = 64 * 197 = 12608 tokens), every tile config, fwd / dgrad /
wgrad (split-K sweep).  Interleaved rounds in one process, min over rounds.
Usage: python scripts/gemm_bench.py [--tokens 12608]"""
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
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) / reps * 1e3)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=12608)
    a = ap.parse_args()
    M = a.tokens
    dev = "cuda"
    cfgs = [c[0] for c in native().gemm_configs()]
    ok = lambda mode, c: native().gemm_config_ok(mode, c)
    print("cfgs:", native().gemm_configs())
    print(f"{'shape':>12} {'pass':>6} {'blas_us':>8} " + " ".join(f"c{c:<7}" for c in cfgs)
          + "  best TF(blas/native)")
    for K, N in [(768, 2304), (768, 768), (768, 3072), (3072, 768)]:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = torch.randn(N, K, device=dev).to(torch.bfloat16)
        b = torch.randn(N, device=dev).to(torch.bfloat16)
        dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        g = torch.zeros(N, K, device=dev)
        fl = 2.0 * M * N * K
        rows = {
            "fwd": (lambda: torch.nn.functional.linear(x, w, b),
                    lambda c: native().gemm(0, 0, c, x, w, y, bias=b)),
            "dgrad": (lambda: dy @ w, lambda c: native().gemm(1, 0, c, dy, w, dx)),
        }
        for name, (blas, nat) in rows.items():
            tb = timeit(blas)
            mode = 0 if name == "fwd" else 1
            ts = {c: (timeit(lambda: nat(c)) if ok(mode, c) else float("nan")) for c in cfgs}
            best = min(v for v in ts.values() if v == v)
            print(f"{K:>5}->{N:<6} {name:>6} {tb:8.1f} " + " ".join(f"{ts[c]:8.1f}" for c in cfgs)
                  + f"  {fl / tb / 1e6:.0f}/{fl / best / 1e6:.0f}", flush=True)
        # wgrad: fp32 accumulate, split-K sweep
        tb = timeit(lambda: torch.ops.aten.addmm.dtype_out(g, dy.t(), x, torch.float32, out=g))
        for slab in (False, True):
            res = {}
            for c in [c for c in cfgs if ok(2, c)]:
                for s in (1, 2, 4, 8, 16):
                    res[(c, s)] = timeit(lambda: native().gemm(2, 3, c, dy, x, g, splits=s,
                                                               slab=slab))
            bestk = min(res, key=res.get)
            tag = "wgradS" if slab else "wgrad"
            print(f"{K:>5}->{N:<6} {tag:>6} {tb:8.1f} "
                  + " ".join(f"{min(res[(c, s)] for s in (1, 2, 4, 8, 16)):8.1f}" if ok(2, c)
                             else "     nan" for c in cfgs)
                  + f"  {fl / tb / 1e6:.0f}/{fl / res[bestk] / 1e6:.0f}  best (cfg, splits)={bestk}",
                  flush=True)
        # slab split-K numerics vs the atomic path
        g1 = torch.zeros_like(g)
        g2 = torch.zeros_like(g)
        native().gemm(2, 3, bestk[0], dy, x, g1, splits=4)
        native().gemm(2, 3, bestk[0], dy, x, g2, splits=4, slab=True)
        err = float((g1 - g2).norm() / g1.norm())
        assert err < 1e-5, err


if __name__ == "__main__":
    main()
