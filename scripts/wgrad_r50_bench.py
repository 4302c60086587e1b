"""3x3 stride-1 weight gradients: every applicable halo wgrad config (atomic and
slab split-K ids) vs the gather kernel's variants, us per call, with a numerics
check of every candidate.  SHAPES=r50 (default: ImageNet ResNet-50 stages 1-2 at
B=128) or SHAPES=r18 (CIFAR ResNet-18 layers at B=512).  Run on the GPU box."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from distributed_ml_pytorch_amd.ops._ext import native
from distributed_ml_pytorch_amd.ops.conv import _wgrad_candidates

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
    which = os.environ.get("SHAPES", "r50")
    r18 = which.startswith("r18")
    st = int(os.environ.get("STRIDE", "1"))
    B = int(os.environ.get("B", "512" if r18 else "128"))
    # (C in, H in, C out); stride 2: the ResNet stride-2 3x3 convs (H in -> H / 2)
    shapes = {"r18": ((64, 32, 64), (128, 16, 128), (256, 8, 256), (512, 4, 512)),
              "r50": ((64, 56, 64), (128, 28, 128), (256, 14, 256), (512, 7, 512)),
              "r18s2": ((64, 32, 128), (128, 16, 256), (256, 8, 512)),
              "r50s2": ((128, 56, 128),)}[which]
    for C, HW, CO in shapes:
        x = torch.randn(B, C, HW, HW, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        OH = HW // st
        dy = torch.randn(B, CO, OH, OH, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        dw = torch.zeros(CO, C, 3, 3, device="cuda").contiguous(memory_format=CL)
        # numerics: every candidate against fp32 autograd of the same conv
        xr = x.float().requires_grad_(False)
        wr = torch.zeros(CO, C, 3, 3, device="cuda", requires_grad=True)
        y = torch.nn.functional.conv2d(xr, wr, None, st, 1)
        y.backward(dy.float())
        ref = wr.grad
        cands = list(nat.conv_wgrad_halo_configs(B, HW, HW, C, CO, 3, 3, st, 1)) + \
            _wgrad_candidates(9 * C, CO)
        res = {}
        for c in cands:
            dw.zero_()
            nat.conv_wgrad(dy, x, dw, st, 1, c)
            err = float((dw - ref).norm() / ref.norm())
            res[c] = (t_us(lambda c=c: nat.conv_wgrad(dy, x, dw, st, 1, c)), err)
        best = min(res, key=lambda c: res[c][0])
        atom = [c for c in res if c < 3000]
        best_atomic = min(atom, key=lambda c: res[c][0])
        tf = 2.0 * B * OH * OH * C * CO * 9 / 1e12
        print(f"C={C} {HW}x{HW} B={B} wgrad best {best} {res[best][0]:.1f} us "
              f"{tf / res[best][0] * 1e6:.0f} TF/s (best without slab: {best_atomic} "
              f"{res[best_atomic][0]:.1f} us) | " +
              " ".join(f"{c}:{u:.0f}({e:.0e})" for c, (u, e) in sorted(res.items())), flush=True)
        assert max(e for _, e in res.values()) < 2e-2


if __name__ == "__main__":
    main()
