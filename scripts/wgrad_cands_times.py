"""Every weight-gradient candidate (gather cfgs, halo cfgs) on the wgrad shapes of one batch
size in the committed tune cache, min of 3 x 10 calls each: the committed pick, the best
overall and the best gather cfg with 512-row pixel chunks per shape.
    python scripts/wgrad_cands_times.py --batch 64"""
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
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    nat = native()
    here = os.path.dirname(os.path.abspath(__file__))
    cache = json.load(open(os.path.join(here, "..", "tuning", "mi355x_tune_cache.json")))
    keys = [json.loads(k) for k in cache if k.startswith('["wgrad", %d,' % a.batch)]
    tot_pick = tot_best = 0.0
    for k in keys:
        _, B, CI, H, W, CO, _, R, S, st, pd = k
        x = torch.randn(B, CI, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        OH, OW = (H + 2 * pd - R) // st + 1, (W + 2 * pd - S) // st + 1
        dy = torch.randn(B, CO, OH, OW, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        dw = torch.zeros(CO, CI, R, S, device="cuda").contiguous(memory_format=CL)
        cands = C._wgrad_candidates(R * S * CI, CO) + list(
            nat.conv_wgrad_halo_configs(B, H, W, CI, CO, R, S, st, pd))
        res = {c: t_us(lambda: nat.conv_wgrad(dy, x, dw, st, pd, c)) for c in cands}
        pick = cache[json.dumps(k)]
        best = min(res.items(), key=lambda kv: kv[1])
        c512 = min(((c, u) for c, u in res.items() if (c >> 4) & 15 == 1 and c < 1000), key=lambda kv: kv[1],
                   default=(None, float("nan")))
        pt = res.get(pick, float("nan"))
        tot_pick += pt if pt == pt else 0.0
        tot_best += best[1]
        print(f"{str(k[1:]):44s} pick {pick}:{pt:6.1f}  best {best[0]}:{best[1]:6.1f}  "
              f"chunk512 {c512[0]}:{c512[1]:6.1f}", flush=True)
    print(f"sum over shapes (one call each): picks {tot_pick:.1f} us, best {tot_best:.1f} us")


if __name__ == "__main__":
    main()
