#!/usr/bin/env python
"""Isolated timing of every GEMM candidate (tile config x split-K, the
any-shape kernel, the skinny weight-gradient kernel) on given shapes: each
candidate called 20x back-to-back inside a hipGraph (launch overhead amortised
as in the training step's graph), no other stream running beside it.

  python scripts/gemm_shape_sweep.py --preset lenet
  python scripts/gemm_shape_sweep.py --shape 2:6:75:50176 --shape 2:120:400:64
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

PRESETS = {
    # (mode, M, N, K): LeNet at bs64 (/root/reference/example/models.py:7-27)
    "lenet": [(2, 6, 75, 50176), (2, 16, 150, 6400), (2, 120, 400, 64), (2, 84, 120, 64),
              (2, 10, 84, 64), (1, 64, 84, 10), (1, 64, 120, 84), (1, 64, 400, 120),
              (1, 6400, 150, 16), (0, 50176, 6, 80), (0, 6400, 16, 152), (0, 64, 120, 400),
              (0, 64, 84, 120), (0, 64, 10, 84)],
    "alexnet": [(2, 64, 363, 4096), (2, 10, 256, 64), (0, 4096, 64, 368), (0, 64, 10, 256),
                (1, 64, 256, 10)],
}


def pad8(v):
    return (v + 7) // 8 * 8


def operands(mode, M, N, K, dev):
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s: torch.randn(*s, device=dev, generator=g).to(torch.bfloat16)  # noqa: E731
    if mode == 2:      # a [K, M], b [K, N] (rows padded to 8 like the arena / im2col operands)
        a = r(K, pad8(M))[:, :M]
        b = r(K, pad8(N))[:, :N]
        c = torch.zeros(M, N, device=dev)
        return a, b, c, 3
    if mode == 1:      # a [M, K], b [K, N]
        a = r(M, pad8(K))[:, :K]
        b = r(K, pad8(N))[:, :N]
    else:              # a [M, K], b [N, K]
        a = r(M, pad8(K))[:, :K]
        b = r(N, pad8(K))[:, :K]
    c = torch.empty(M, pad8(N), device=dev, dtype=torch.bfloat16)[:, :N]
    return a, b, c, 0


def time_fn(fn, reps=50, chain=20):
    """Median per-call time of ``chain`` back-to-back calls replayed from a
    hipGraph (the in-graph condition: no host launch gap between kernels)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            for _ in range(chain):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    fn = graph.replay
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
    for i in range(reps):
        ev[2 * i].record()
        fn()
        ev[2 * i + 1].record()
    torch.cuda.synchronize()
    ts = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) * 1e3 for i in range(reps))
    return ts[len(ts) // 2] / chain


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", action="append", default=[])
    ap.add_argument("--shape", action="append", default=[], help="mode:M:N:K")
    ap.add_argument("--top", type=int, default=4)
    args = ap.parse_args()
    from distributed_ml_pytorch_amd.ops import linear as LIN
    from distributed_ml_pytorch_amd.ops._ext import native

    shapes = [s for p in args.preset for s in PRESETS[p]]
    shapes += [tuple(int(v) for v in s.split(":")) for s in args.shape]
    dev = torch.device("cuda")
    nat = native()
    for mode, M, N, K in shapes:
        a, b, c, epi = operands(mode, M, N, K, dev)
        ok = LIN._mfma_ok(mode, M, N, K, a, b)
        cands = LIN._candidates(mode, epi, M, N, K, True, ok)
        res = []
        for e in cands:
            if e == LIN._BLAS:
                continue
            if e == LIN._SKINNY:
                fn = lambda: nat.gemm(mode, epi, -2, a, b, c, None, None, None, None, 1,  # noqa
                                      False, None, False)
                name = "skinny"
            else:
                cfg, sp = LIN._dec(e)
                slab = LIN._dec_slab(e)
                fn = (lambda cfg=cfg, sp=sp, slab=slab: nat.gemm(
                    mode, epi, cfg, a, b, c, None, None, None, None, sp, False, None, slab))
                name = f"cfg{cfg}x{sp}{'s' if slab else ''}"
            try:
                res.append((time_fn(fn), name))
            except RuntimeError as ex:      # a candidate the launcher refuses
                res.append((float("inf"), f"{name}:{str(ex)[:40]}"))
        res.sort()
        shown = res[:args.top] + [r for r in res[args.top:] if r[1] == "skinny"]
        best = ", ".join(f"{n} {t:.1f}" for t, n in shown)
        print(f"mode {mode} M {M:6d} N {N:5d} K {K:6d} mfma_ok {int(ok)} "
              f"({len(res)} cands) us: {best}", flush=True)


if __name__ == "__main__":
    main()
