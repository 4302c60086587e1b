"""Time the folded BatchNorm backward (bn_bwd_fold: two launches, or the one-pass
kernel with DMP_BN_BWD_ONEPASS=1) at the ResNet-18 bs512 shapes; the env knob is
read once per process: DMP_BN_BWD_ONEPASS=0 python scripts/bn_bwd_one.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_ml_pytorch_amd.ops._ext import native  # noqa: E402


def main():
    nat = native()
    CL = torch.channels_last
    tag = os.environ.get("DMP_BN_BWD_ONEPASS", "1")
    for B, C, H in ((512, 64, 32), (512, 128, 16), (512, 256, 8), (512, 512, 4)):
        x = torch.randn(B, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        dy = torch.randn_like(x)
        gamma = torch.rand(C, device="cuda") + 0.5
        stats = torch.cat([torch.zeros(C, device="cuda"), torch.ones(C, device="cuda"),
                           gamma, torch.zeros(C, device="cuda")])
        mask = torch.randint(0, 256, (B * H * H * C // 8,), device="cuda", dtype=torch.uint8)
        slots = torch.zeros(2 * 64 * C + 4, device="cuda")
        zb = torch.zeros_like(slots)
        dg = torch.zeros(C, device="cuda")
        db = torch.zeros(C, device="cuda")
        for mode in (2, 3):
            def run():
                nat.bn_bwd_fold(x, dy, None, gamma, stats, dg, db, True, False, slots,
                                mask if mode == 3 else None, zb)
            run()
            torch.cuda.synchronize()
            ts = []
            for _ in range(7):
                a = torch.cuda.Event(enable_timing=True)
                b = torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(20):
                    run()
                b.record()
                b.synchronize()
                ts.append(a.elapsed_time(b) / 20 * 1e3)
            ts.sort()
            print(f"onepass={tag} B={B} C={C} H={H} mode={mode}: {ts[len(ts) // 2]:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
