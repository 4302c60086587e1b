"""ViT-B/16 MLP GEMMs with their fused epilogues, every tile config: fc1 forward
with the GELU epilogue (h and gelu(h) stored) and fc2 data gradient with the
GELU' epilogue (reads h), next to the plain store epilogue of the same GEMM.
us per call (min over rounds).  Run on the GPU box."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from distributed_ml_pytorch_amd.ops._ext import native


def timeit(fn, it=10, rounds=3):
    fn()
    best = float("inf")
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(it):
            fn()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / it)
    return best


def main():
    nat = native()
    M, D, F = 12608, 768, 3072
    dev = "cuda"
    x = torch.randn(M, D, device=dev).to(torch.bfloat16)
    w1 = (torch.randn(F, D, device=dev) * 0.02).to(torch.bfloat16)
    b1 = torch.zeros(F, device=dev).to(torch.bfloat16)
    h = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    a = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(M, D, device=dev).to(torch.bfloat16)
    w2 = (torch.randn(D, F, device=dev) * 0.02).to(torch.bfloat16)
    da = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * M * D * F
    cfgs = [c[0] for c in nat.gemm_configs()]
    rows = {
        "fc1 fwd store": (0, lambda c: nat.gemm(0, 0, c, x, w1, h, bias=b1)),
        "fc1 fwd GELU ": (0, lambda c: nat.gemm(0, 1, c, x, w1, h, a, bias=b1)),
        "fc2 dgrad    ": (1, lambda c: nat.gemm(1, 0, c, dy, w2, da)),
        "fc2 dgrad dGELU": (1, lambda c: nat.gemm(1, 2, c, dy, w2, da, aux=h)),
    }
    print("cfgs:", nat.gemm_configs())
    for name, (mode, run) in rows.items():
        ts = {c: timeit(lambda c=c: run(c)) for c in cfgs if nat.gemm_config_ok(mode, c)}
        best = min(ts, key=ts.get)
        print(f"{name:16s} best cfg {best}: {ts[best]:6.1f} us {fl / ts[best] / 1e6:5.0f} TF/s | "
              + " ".join(f"{c}:{t:.0f}" for c, t in sorted(ts.items())), flush=True)


if __name__ == "__main__":
    main()
