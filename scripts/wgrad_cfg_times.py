"""Per-config times (us, min of 3x10) of every halo weight-gradient config (atomic ids
1000+, slab ids 3000+) on the ResNet-18 CIFAR 3x3 stride-1 layers at the bench batch,
plus the tune-cache pick.  Used for A/B runs of csrc/conv_wgrad.hip (run the same
script against two builds)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.environ.get("DMP_AB_ROOT", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")))
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
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    nat = native()
    here = os.path.dirname(os.path.abspath(__file__))
    cache = json.load(open(os.path.join(here, "..", "tuning", "mi355x_tune_cache.json")))
    for C, HW in ((64, 32), (128, 16), (256, 8), (512, 4)):
        B = a.batch
        x = torch.randn(B, C, HW, HW, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        dy = torch.randn(B, C, HW, HW, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        dw = torch.zeros(C, C, 3, 3, device="cuda").contiguous(memory_format=CL)
        slab = None
        tf = 2.0 * B * HW * HW * C * C * 9 / 1e12
        res = {}
        for c in nat.conv_wgrad_halo_configs(B, HW, HW, C, C, 3, 3, 1, 1):
            res[c] = t_us(lambda: nat.conv_wgrad(dy, x, dw, 1, 1, c))
        pick = cache.get(json.dumps(["wgrad", B, C, HW, HW, C, C, 3, 3, 1, 1]))
        top = sorted(res.items(), key=lambda kv: kv[1])[:6]
        print(f"{a.tag} C={C:3d} {HW}x{HW}: pick {pick} {res.get(pick, float('nan')):6.1f} us | best " +
              " ".join(f"{c}:{u:.1f}" for c, u in top) +
              f" | {tf / top[0][1] * 1e6:.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
