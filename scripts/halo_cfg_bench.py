"""Every halo-tile config (csrc/conv.hip DMP_HALO_CONFIGS) on the ResNet-18 CIFAR
3x3 stride-1 layers: forward (+BN partial sums) and data gradient, us per call
(min over rounds) and TF/s of the best.  Run on the GPU box."""
import argparse
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
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--shapes", default="r18", choices=["r18", "r50"],
                    help="r18: CIFAR ResNet-18 layers; r50: ImageNet ResNet-50 3x3 stride-1 convs "
                         "(14x14 / 7x7: padded whole-image tiles)")
    ap.add_argument("--igemm", type=int, default=0, help="also time the implicit-GEMM tiles")
    a = ap.parse_args()
    nat = native()
    shapes = ((64, 32), (128, 16), (256, 8), (512, 4)) if a.shapes == "r18" else \
        ((64, 56), (128, 28), (256, 14), (512, 7))
    for C, HW in shapes:
        B = a.batch
        x = torch.randn(B, C, HW, HW, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        w = (torch.randn(C, C, 3, 3, device="cuda") * 0.02).to(torch.bfloat16).contiguous(memory_format=CL)
        dy = torch.randn(B, C, HW, HW, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        tf = 2.0 * B * HW * HW * C * C * 9 / 1e12
        for name, run in (("fwd", lambda c: nat.conv_fwd(x, w, 1, 1, True, c)),
                          ("dgrad", lambda c: nat.conv_dgrad(dy, w, HW, HW, 1, 1, c))):
            cands = list(nat.conv_halo_configs(HW, HW, C, 3, 3, 1, 1))
            if a.igemm:
                cands += list(range(nat.conv_num_configs() if hasattr(nat, "conv_num_configs")
                                    else len(nat.conv_configs())))
            ref = run(-1)[0] if name == "fwd" else run(-1)
            res = {}
            for c in cands:
                out = run(c)
                out = out[0] if name == "fwd" else out
                err = float((out.float() - ref.float()).abs().max() / ref.float().abs().max())
                if not err < 2e-2:
                    print(f"  cfg {c}: MISMATCH rel err {err:.3e}", flush=True)
                    continue
                res[c] = t_us(lambda c=c: run(c))
            best = min(res, key=res.get)
            print(f"C={C:3d} {HW:2d}x{HW:<2d} {name:5s} best {best} {res[best]:6.1f} us "
                  f"{tf / res[best] * 1e6:5.0f} TF/s | " +
                  " ".join(f"{c}:{u:.0f}" for c, u in sorted(res.items())), flush=True)


if __name__ == "__main__":
    main()
