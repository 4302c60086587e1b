"""ResNet-50 bs128 1x1 forward convs (+BN partial sums): every implicit-GEMM conv
tile vs every GEMM-route tile (csrc/gemm.hip, stats epilogue), us per call, and the
HBM roofline of the layer (input + output bytes at 6 TB/s)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from distributed_ml_pytorch_amd.ops._ext import native  # noqa: E402
from distributed_ml_pytorch_amd.ops.conv import BN_SLOTS, BN_TAIL  # noqa: E402

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
    B = 128
    for CI, HW, CO in ((64, 56, 256), (256, 56, 64), (64, 56, 64), (128, 28, 512), (512, 28, 128),
                       (256, 14, 1024), (1024, 14, 256), (512, 7, 2048), (2048, 7, 512)):
        x = torch.randn(B, CI, HW, HW, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        w = (torch.randn(CO, CI, 1, 1, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=CL)
        M = B * HW * HW
        x2 = x.permute(0, 2, 3, 1).reshape(M, CI)
        y2 = torch.empty(M, CO, dtype=torch.bfloat16, device="cuda")
        part = torch.zeros(2 * BN_SLOTS * CO + BN_TAIL, device="cuda")
        res = {}
        for c in range(len(nat.conv_configs())):
            res[f"c{c}"] = t_us(lambda c=c: nat.conv_fwd(x, w, 1, 0, True, c))
        for g in nat.gemm_configs():
            cid = g[0]
            if not nat.gemm_config_ok(0, cid):
                continue
            res[f"g{cid}"] = t_us(lambda cid=cid: nat.gemm(0, 0, cid, x2, w.reshape(CO, CI), y2,
                                                           part=part))
        roof = (M * (CI + CO) * 2) / 6e12 * 1e6
        bi = min((k for k in res if k[0] == "c"), key=res.get)
        bg = min((k for k in res if k[0] == "g"), key=res.get)
        print(f"{CI:4d}->{CO:4d} {HW}x{HW}: conv {bi} {res[bi]:.1f} us | gemm {bg} {res[bg]:.1f} us | "
              f"HBM roofline {roof:.1f} us | " + " ".join(f"{k}:{v:.0f}" for k, v in res.items()),
              flush=True)


if __name__ == "__main__":
    main()
