"""3x3 / stride-2 forward on the ResNet-18 stride-2 layers (B=512): every
stride-2 halo config vs every implicit-GEMM tile, us per call (min over rounds)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from distributed_ml_pytorch_amd.ops._ext import native  # noqa: E402

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
    B = int(os.environ.get("B", "512"))
    for C, H, CO in ((64, 32, 128), (128, 16, 256), (256, 8, 512)):
        x = torch.randn(B, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        w = (torch.randn(CO, C, 3, 3, device="cuda") * 0.02).to(torch.bfloat16).contiguous(memory_format=CL)
        ref = nat.conv_fwd(x, w, 2, 1, True, -1)[0].float()
        cands = list(nat.conv_halo_configs(H, H, C, 3, 3, 2, 1)) + list(range(len(nat.conv_configs())))
        res = {}
        for c in cands:
            y = nat.conv_fwd(x, w, 2, 1, True, c)[0].float()
            if not float((y - ref).abs().max() / ref.abs().max()) < 2e-2:
                print(f"  cfg {c}: MISMATCH", flush=True)
                continue
            res[c] = t_us(lambda c=c: nat.conv_fwd(x, w, 2, 1, True, c))
        tf = 2.0 * B * (H // 2) ** 2 * C * CO * 9 / 1e12
        best = min(res, key=res.get)
        halo = {c: v for c, v in res.items() if c >= 100}
        bh = min(halo, key=halo.get) if halo else None
        ig = {c: v for c, v in res.items() if c < 100}
        bi = min(ig, key=ig.get)
        print(f"{C}->{CO} {H}x{H} s2 fwd: best {best} {res[best]:.1f} us {tf / res[best] * 1e6:.0f} TF/s; "
              f"halo {bh} {halo.get(bh, float('nan')):.1f} us, igemm {bi} {ig[bi]:.1f} us | "
              + " ".join(f"{c}:{v:.0f}" for c, v in sorted(res.items())), flush=True)


if __name__ == "__main__":
    main()
