"""Time the CIFAR stem kernels (conv_small.hip stem3_fwd / stem3_wgrad) at the
ResNet-18 bs512 shape in one process; the launch knobs DMP_STEM3_GROUPS /
DMP_STEM3_WG_BLOCKS are read once per process, so sweep them across runs:
for g in 16 8 4; do DMP_STEM3_GROUPS=$g python scripts/stem3_one.py; done"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_ml_pytorch_amd.ops._ext import native  # noqa: E402


def timeit(fn, reps=20, rounds=7):
    best = []
    for _ in range(rounds):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        b.synchronize()
        best.append(a.elapsed_time(b) / reps * 1e3)
    best.sort()
    return best[len(best) // 2]


def main():
    CL = torch.channels_last
    B = int(os.environ.get("STEM_B", "512"))
    x = torch.randn(B, 3, 32, 32, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    w = (0.2 * torch.randn(64, 3, 3, 3, device="cuda")).to(torch.bfloat16).contiguous(memory_format=CL)
    dy = torch.randn(B, 64, 32, 32, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    dw = torch.zeros(64, 3, 3, 3, device="cuda").contiguous(memory_format=CL)
    nat = native()
    slots = torch.zeros(2 * 64 * 64 + 4, device="cuda")

    def fwd():
        nat.conv_small_fwd(x, w, 1, 1, True, slots)

    def wg():
        nat.conv_small_wgrad(dy, x, dw, 1, 1)
    fwd(); wg(); torch.cuda.synchronize()
    print(f"pf={os.environ.get('DMP_STEM3_PF', '2')} groups={os.environ.get('DMP_STEM3_GROUPS', '16')} wg_blocks="
          f"{os.environ.get('DMP_STEM3_WG_BLOCKS', '512')}  fwd {timeit(fwd):6.1f} us  "
          f"wgrad {timeit(wg):6.1f} us", flush=True)


if __name__ == "__main__":
    main()
