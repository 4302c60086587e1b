"""3x3 / stride-2 data gradient: every stride-2 halo config (conv_dgrad_s2_kernel) and
every implicit-GEMM tile on the ResNet-18 CIFAR (B=512) and ResNet-50 stage-2 (B=128)
stride-2 layers; us per call (min of 3x10), TF/s of the best, and the tune-cache pick."""
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
    nat = native()
    here = os.path.dirname(os.path.abspath(__file__))
    cache = json.load(open(os.path.join(here, "..", "tuning", "mi355x_tune_cache.json")))
    for B, CI, H, CO in ((512, 64, 32, 128), (512, 128, 16, 256), (512, 256, 8, 512),
                         (128, 128, 56, 128)):
        OH = H // 2
        w = (torch.randn(CO, CI, 3, 3, device="cuda") * 0.02).to(torch.bfloat16).contiguous(memory_format=CL)
        dy = torch.randn(B, CO, OH, OH, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        tf = 2.0 * B * OH * OH * CO * CI * 9 / 1e12
        res = {}
        for c in list(nat.conv_dgrad_s2_configs(H, H, OH, OH, CO, CI, 3, 3, 2, 1)) + \
                [c[0] for c in nat.conv_configs()]:
            res[c] = t_us(lambda c=c: nat.conv_dgrad(dy, w, H, H, 2, 1, c))
        key = json.dumps(["dgrad", B, CO, OH, OH, CI, H, H, 3, 3, 2, 1])
        pick = cache.get(key)
        best = min(res, key=res.get)
        s2 = {c: u for c, u in res.items() if c >= 200}
        print(f"B{B} {CI}<-{CO} {H}x{H} s2: cache pick {pick} {res.get(pick, float('nan')):6.1f} us | "
              f"best {best} {res[best]:6.1f} us {tf / res[best] * 1e6:5.0f} TF/s | s2 " +
              " ".join(f"{c}:{u:.1f}" for c, u in sorted(s2.items())) +
              " | igemm best " + str(min((u, c) for c, u in res.items() if c < 200)), flush=True)


if __name__ == "__main__":
    main()
