"""Every forward / data-gradient (/ weight-gradient with --kinds) candidate the tuner offers
(ops/conv.py _fwd_cfg / _dgrad_cfg / _wgrad_cfg) on the
conv shapes of one batch size in the committed tune cache, min of 3 x 10 calls each: the committed pick
and the best candidate per key, and a candidate cache (committed picks, with every key whose best is
more than --margin faster replaced) for an in-step A/B.
    python scripts/conv_cands_times.py --batch 64 --out gpurun_out/cand_fwd_dgrad.json"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from distributed_ml_pytorch_amd.ops import conv as C
from distributed_ml_pytorch_amd.ops._ext import native

CL = torch.channels_last


def t_us(fn, it=10, rounds=3):
    """Per-call device time of ``fn`` replayed from a captured graph (as in the training
    step: a Python-side route's host cost does not count), min over ``rounds``."""
    fn()                                   # first call: any inner GEMM pick is tuned here
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(it):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / it)
    del g
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--margin", type=float, default=0.05)
    ap.add_argument("--out", default="gpurun_out/cand_fwd_dgrad.json")
    ap.add_argument("--kinds", default="fwd,dgrad", help="comma list of fwd / dgrad / wgrad")
    a = ap.parse_args()
    nat = native()
    here = os.path.dirname(os.path.abspath(__file__))
    path = os.path.join(here, "..", "tuning", "mi355x_tune_cache.json")
    cache = json.load(open(path))
    cand = dict(cache)
    # the GEMM routes' inner GEMMs: committed picks, new keys tuned on first use
    from distributed_ml_pytorch_amd.ops.tuner import TUNER
    TUNER.cache.update({tuple(json.loads(ks)): v for ks, v in cache.items()})
    for ks, pick in cache.items():
        k = json.loads(ks)
        if k[0] not in a.kinds.split(",") or k[1] != a.batch:
            continue
        if k[0] == "wgrad":
            _, B, CI, H, W, CO, _ci, R, S, st, pd = k
            OH, OW = (H + 2 * pd - R) // st + 1, (W + 2 * pd - S) // st + 1
        elif k[0] == "fwd":
            _, B, CI, H, W, CO, R, S, st, pd = k
            OH, OW = (H + 2 * pd - R) // st + 1, (W + 2 * pd - S) // st + 1
        else:
            _, B, CO, OH, OW, CI, H, W, R, S, st, pd = k
        if CI % 8 or CO % 64:
            continue                      # the small-CI stems have their own kernels
        x = torch.randn(B, CI, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        w = (torch.randn(CO, CI, R, S, device="cuda") / (R * S * CI) ** 0.5).to(torch.bfloat16).contiguous(
            memory_format=CL)
        dy = torch.randn(B, CO, OH, OW, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        if k[0] == "wgrad":
            dw = torch.zeros(CO, CI, R, S, device="cuda").contiguous(memory_format=CL)
            cands = C._wgrad_candidates(R * S * CI, CO) + list(
                nat.conv_wgrad_halo_configs(B, H, W, CI, CO, R, S, st, pd))
            if C._gemm1x1_ok((CO, CI, R, S), st, pd, CI, CO):
                cands.append(C._GEMM_ROUTE)
            elif C._im2col_wgrad_ok(x, (CO, CI, R, S), st, pd):
                cands.append(C._IM2COL_ROUTE)
            run = lambda c: (C._gemm_route_wgrad(c, dy, x, dw, st, pd)   # noqa: E731
                             if c in (C._GEMM_ROUTE, C._IM2COL_ROUTE)
                             else nat.conv_wgrad(dy, x, dw, st, pd, c))
        elif k[0] == "fwd":
            cands = C._igemm_candidates(CO) + C._halo_candidates(H, W, CI, R, S, st, pd)
            run = lambda c: nat.conv_fwd(x, w, st, pd, True, c)   # noqa: E731
        else:
            cands = C._igemm_candidates(CI, fwd=st == 1)
            if (H, W) == (OH, OW):
                cands += C._halo_candidates(H, W, CO, R, S, st, pd)
            elif st == 2:
                cands += list(nat.conv_dgrad_s2_configs(H, W, OH, OW, CO, CI, R, S, st, pd))
            run = lambda c: nat.conv_dgrad(dy, w, H, W, st, pd, c)   # noqa: E731
        res = {}
        for c in cands:
            try:
                res[c] = t_us(lambda: run(c))
            except RuntimeError as e:
                if c >= C._GEMM_ROUTE:
                    print(f"  route {c} failed: {e}", flush=True)
        best = min(res.items(), key=lambda kv: kv[1])
        pt = res.get(pick, float("nan"))
        flag = ""
        if pt == pt and best[1] < (1 - a.margin) * pt:
            cand[ks] = best[0]
            flag = "  <- candidate"
        route = next((f"  route {c}:{res.get(c, float('nan')):6.1f}" for c in
                      (C._GEMM_ROUTE, C._IM2COL_ROUTE) if c in cands), "")
        print(f"{str(k):58s} pick {pick}:{pt:6.1f}  best {best[0]}:{best[1]:6.1f}{route}{flag}",
              flush=True)
    for kt, v in TUNER.cache.items():          # GEMM keys first tuned here
        ks = json.dumps(list(kt))
        if ks not in cand and kt[0] == "gemm":
            cand[ks] = v
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(cand, open(a.out, "w"), indent=0, sort_keys=True)


if __name__ == "__main__":
    main()
