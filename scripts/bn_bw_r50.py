"""Achieved HBM bandwidth of the folded BatchNorm kernels at the ResNet-50 bs128
shapes (VERDICT r5 #3 pricing): forward apply (ReLU; residual + ReLU + 1-bit mask)
and the backward pair (bn_partial_kernel reduce + bn_bwd_apply_fold_kernel), each
timed per kernel under torch.profiler, bytes = the tensors each kernel must stream.

    python scripts/bn_bw_r50.py [--batch 128]
"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from distributed_ml_pytorch_amd.ops._ext import native  # noqa: E402

# (channels, spatial) of every distinct BN tensor of ResNet-50 at 224^2, with the
# number of BN layers of that shape per step (bn1/bn2 inner, bn3 + shortcut outer)
SHAPES = [(64, 56, 6), (256, 56, 4), (128, 56, 1), (128, 28, 7), (512, 28, 5),
          (256, 28, 1), (256, 14, 11), (1024, 14, 7), (512, 14, 1), (512, 7, 5),
          (2048, 7, 4)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    nat = native()
    CL = torch.channels_last
    tot = collections.Counter()
    print(f"{'C':>5} {'HxW':>6} {'n':>2} {'MB':>7} | {'kernel':<26} {'us':>7} {'TB/s':>6}")
    for C, H, n in SHAPES:
        B = a.batch
        x = torch.randn(B, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        res = torch.randn_like(x)
        dy = torch.randn_like(x)
        S = x.numel() * 2
        gamma = torch.rand(C, device="cuda") + 0.5
        beta = torch.randn(C, device="cuda") * 0.1
        slots = torch.zeros(2 * 64 * C + 4, device="cuda")
        zb = torch.zeros_like(slots)
        M = x.numel() // C

        def fill_fwd_slots():   # the producing conv's epilogue sums (one slot row)
            xs = x.float().reshape(M, C)
            slots[:C] = xs.sum(0)
            slots[64 * C:65 * C] = (xs * xs).sum(0)

        fill_fwd_slots()
        # warm: compile paths + a stats tensor for the backward
        y, stats, mask = nat.bn_fwd_fold(x, slots, True, res, gamma, beta, None, None, 0.1, 1e-5,
                                         True, True, zb)
        dg = torch.zeros(C, device="cuda")
        db = torch.zeros(C, device="cuda")
        bslots = torch.zeros_like(slots)
        arms = {
            "fwd relu": lambda: nat.bn_fwd_fold(x, slots, True, None, gamma, beta, None, None, 0.1,
                                                1e-5, True, False, zb),
            "fwd res+relu+mask": lambda: nat.bn_fwd_fold(x, slots, True, res, gamma, beta, None,
                                                         None, 0.1, 1e-5, True, True, zb),
            "bwd relu(x)": lambda: nat.bn_bwd_fold(x, dy, None, gamma, stats, dg, db, True, False,
                                                   bslots, None, zb),
            "bwd mask": lambda: nat.bn_bwd_fold(x, dy, None, gamma, stats, dg, db, True, False,
                                                bslots, mask, zb),
        }
        bytes_of = {"bn_apply_fold_kernel<64, true, false": 2 * S,
                    "bn_apply_fold_kernel<64, true, true": 3 * S + S // 16,
                    "bn_partial_kernel<1, 2>": 2 * S, "bn_partial_kernel<1, 3>": 2 * S + S // 16,
                    "bn_bwd_apply_fold_kernel<64, 2": 3 * S,
                    "bn_bwd_apply_fold_kernel<64, 3": 3 * S + S // 16}
        for name, fn in arms.items():
            fn()
            torch.cuda.synchronize()
            with profile(activities=[ProfilerActivity.CUDA]) as prof:
                for _ in range(a.reps):
                    fn()
                torch.cuda.synchronize()
            agg = collections.defaultdict(float)
            for e in prof.events():
                if e.device_type == torch.autograd.DeviceType.CUDA and "dmp::" in e.name:
                    agg[e.name] += e.device_time / a.reps
            for kn, us in sorted(agg.items()):
                short = kn.replace("void dmp::", "")
                key = next((k for k in bytes_of if k in short), None)
                bw = f"{bytes_of[key] / us / 1e6:6.2f}" if key else "     -"
                print(f"{C:5d} {H:3d}x{H:<2d} {n:2d} {S / 1e6:7.1f} | {name:<18} {short[:44]:<44} "
                      f"{us:7.1f} {bw}", flush=True)
                tot[name] += us * n
        del x, res, dy, y, mask
        torch.cuda.empty_cache()
    print("per-step totals if every BN of the shape ran this arm (us):",
          {k: round(v, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
