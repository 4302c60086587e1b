"""Every GEMM candidate the tuner offers (ops/linear.py _candidates) on the GEMM keys of the committed
tune cache whose M is --m (ViT-B/16 bs64: 12608 tokens), min of 3 x 10 calls each, the committed pick
next to the best; keys whose best beats the pick by more than --margin are swapped into a candidate
cache for an in-step A/B.
    python scripts/gemm_cands_times.py --m 12608 --out gpurun_out/cand_gemm.json"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from distributed_ml_pytorch_amd.ops import linear as L
from distributed_ml_pytorch_amd.ops._ext import native


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=12608)
    ap.add_argument("--margin", type=float, default=0.03)
    ap.add_argument("--out", default="gpurun_out/cand_gemm.json")
    a = ap.parse_args()
    nat = native()
    here = os.path.dirname(os.path.abspath(__file__))
    cache = json.load(open(os.path.join(here, "..", "tuning", "mi355x_tune_cache.json")))
    cand = dict(cache)
    bf = dict(device="cuda", dtype=torch.bfloat16)
    for ks, pick in cache.items():
        k = json.loads(ks)
        if k[0] != "gemm":
            continue
        mode, epi, M, N, K, has_bias, has_aux, has_db, relu = k[1:10]
        if a.m not in (M, K) or len(k) > 10:
            continue
        if mode == 2:
            A = torch.randn(K, M, **bf)
            B = torch.randn(K, N, **bf)
            Cc = torch.zeros(M, N, device="cuda")
        else:
            A = torch.randn(M, K, **bf)
            B = torch.randn(N, K, **bf) if mode == 0 else torch.randn(K, N, **bf)
            Cc = torch.empty(M, N, **bf)
        C2 = torch.empty(M, N, **bf) if epi == 1 else None
        bias = torch.randn(N, **bf) if has_bias else None
        aux = torch.randn(M, N, **bf) if has_aux else None
        db = torch.zeros(M, device="cuda") if has_db else None
        cands = L._candidates(mode, epi, M, N, K, True)
        res = {}
        for e in cands:
            cfg, sp = L._dec(e)
            try:
                res[e] = t_us(lambda: nat.gemm(mode, epi, cfg, A, B, Cc, C2, bias, aux, db, sp, relu,
                                               None, L._dec_slab(e)))
            except RuntimeError:
                pass
        best = min(res.items(), key=lambda kv: kv[1])
        pt = res.get(pick, float("nan"))
        flag = ""
        if pt == pt and best[1] < (1 - a.margin) * pt:
            cand[ks] = best[0]
            flag = "  <- candidate"
        print(f"{str(k[1:]):50s} pick {pick}:{pt:7.1f}  best {best[0]}:{best[1]:7.1f}{flag}", flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(cand, open(a.out, "w"), indent=0, sort_keys=True)


if __name__ == "__main__":
    main()
