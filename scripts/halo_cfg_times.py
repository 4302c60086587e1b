"""Per-config times (us, min of 3 x 10 calls) of every 3x3 stride-1 halo forward / data-gradient
config on the ResNet-18 layers at one batch size, next to the committed tune-cache pick.
    python scripts/halo_cfg_times.py --batch 64"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

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
    B = a.batch
    for C, H in ((64, 32), (128, 16), (256, 8), (512, 4)):
        x = torch.randn(B, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        w = (torch.randn(C, C, 3, 3, device="cuda") / (9 * C) ** 0.5).to(torch.bfloat16).contiguous(
            memory_format=CL)
        dy = torch.randn_like(x)
        cfgs = list(nat.conv_halo_configs(H, H, C, 3, 3, 1, 1))
        fwd = {c: t_us(lambda: nat.conv_fwd(x, w, 1, 1, True, c)) for c in cfgs}
        dgr = {c: t_us(lambda: nat.conv_dgrad(dy, w, H, H, 1, 1, c)) for c in cfgs}
        pf = cache.get(json.dumps(["fwd", B, C, H, H, C, 3, 3, 1, 1]))
        pd = cache.get(json.dumps(["dgrad", B, C, H, H, C, H, H, 3, 3, 1, 1]))
        for name, res, pick in (("fwd", fwd, pf), ("dgrad", dgr, pd)):
            top = sorted(res.items(), key=lambda kv: kv[1])[:5]
            new = {c: round(res[c], 1) for c in (126, 127) if c in res}
            print(f"C={C:3d} {H}x{H} {name:5s} pick {pick}:{res.get(pick, float('nan')):6.1f} | best "
                  + " ".join(f"{c}:{u:.1f}" for c, u in top) + f" | ns3 {new}", flush=True)


if __name__ == "__main__":
    main()
