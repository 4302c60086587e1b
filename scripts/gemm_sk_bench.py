"""Remainder split-K (csrc/gemm.hip GemmArgs sk_*) on the ViT-B/16 fwd / dgrad
GEMMs (bs64: M = 12608 tokens) against the unsplit tiles and hipBLASLt.

For every tile config the unsplit launch and the splits the plan accepts (2, 4)
are timed in interleaved rounds in one process (min over rounds); hipBLASLt =
torch.nn.functional.linear / matmul on the same operands.  Usage:
python scripts/gemm_sk_bench.py [--tokens 12608]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_ml_pytorch_amd.ops._ext import native  # noqa: E402


def timeit(fn, reps=10):
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=12608)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    M = args.tokens
    dev = "cuda"
    cfgs = [c[0] for c in native().gemm_configs() if c[0] <= 8 or c[0] >= 10]
    print("cfgs:", [c for c in native().gemm_configs() if c[0] in cfgs])
    for K, N in [(768, 2304), (768, 768), (768, 3072), (3072, 768)]:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = torch.randn(N, K, device=dev).to(torch.bfloat16)
        bias = torch.randn(N, device=dev).to(torch.bfloat16)
        dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        for name, mode in (("fwd", 0), ("dgrad", 1)):
            arms = {"blas": (lambda: torch.nn.functional.linear(x, w, bias)) if mode == 0
                    else (lambda: dy @ w)}
            outN = N if mode == 0 else K
            for c in cfgs:
                if not native().gemm_config_ok(mode, c):
                    continue
                for s in (1, 2, 4):
                    if s > 1 and native().gemm_sk_pieces(c, M, outN, K if mode == 0 else N, s) <= 0:
                        continue
                    if mode == 0:
                        arms[(c, s)] = (lambda c=c, s=s:
                                        native().gemm(0, 0, c, x, w, y, bias=bias, splits=s))
                    else:
                        arms[(c, s)] = (lambda c=c, s=s: native().gemm(1, 0, c, dy, w, dx, splits=s))
            for fn in arms.values():
                fn()
            torch.cuda.synchronize()
            best = {k: float("inf") for k in arms}
            for _ in range(args.rounds):
                for k, fn in arms.items():
                    best[k] = min(best[k], timeit(fn))
            tb = best.pop("blas")
            unsplit = {k: v for k, v in best.items() if k[1] == 1}
            split = {k: v for k, v in best.items() if k[1] > 1}
            b1 = min(unsplit, key=unsplit.get)
            line = (f"{K:>5}->{N:<5} {name:>5}  hipBLASLt {tb:6.1f}  best unsplit {unsplit[b1]:6.1f} "
                    f"(c{b1[0]})")
            if split:
                b2 = min(split, key=split.get)
                line += f"  best split-K {split[b2]:6.1f} (c{b2[0]} s{b2[1]})"
                base = unsplit.get((b2[0], 1), float("nan"))
                line += f" [same cfg unsplit {base:6.1f}]"
            allbest = min(best.values())
            line += f"  TF/s blas {fl / tb / 1e6:.0f} / native {fl / allbest / 1e6:.0f}"
            print(line, flush=True)
            for k in sorted(split):
                print(f"      c{k[0]} s{k[1]}: {split[k]:6.1f} us  (unsplit {unsplit.get((k[0], 1), float('nan')):6.1f})")


if __name__ == "__main__":
    main()
