"""Whole-model gradient parity + short training trajectory, native framework vs stock
PyTorch on identical weights and data (GPU).  Prints per-parameter relative gradient
error of (a) our native bf16 step and (b) stock autocast-bf16, both against stock fp32,
then the loss trajectory of plain SGD for both implementations.

    python scripts/grad_parity.py --model resnet18 --batch 256 --steps 40
"""
from __future__ import annotations

import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import stock_baseline as sb  # noqa: E402

from distributed_ml_pytorch_amd.runtime.dist import DistInfo  # noqa: E402
from distributed_ml_pytorch_amd.runtime.trainer import TrainConfig, Worker  # noqa: E402


def rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--zero-init-residual", action="store_true",
                    help="zero the last BatchNorm gamma of every residual block (both models): "
                         "the well-conditioned start where stock bf16 is itself close to fp32")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    mk = lambda lr: Worker(TrainConfig(model=a.model, batch_size=a.batch, mode="single", lr=lr,  # noqa: E731
                                       evaluate=False, verbose=False), DistInfo(device=dev))
    def zero_res(worker):
        if not a.zero_init_residual:
            return
        from distributed_ml_pytorch_amd.models.resnet import BasicBlock, Bottleneck

        with torch.no_grad():
            for m in worker.model.modules():
                if isinstance(m, Bottleneck):
                    m.bn3.weight.zero_()
                elif isinstance(m, BasicBlock):
                    m.bn2.weight.zero_()
        worker.arena.refresh_shadow()

    w = mk(0.0)
    zero_res(w)
    ctor, shape, nc = sb.MODELS[a.model]
    ref = ctor().to(dev).to(memory_format=torch.channels_last)
    P, Q = list(w.model.parameters()), list(ref.parameters())
    assert len(P) == len(Q)
    with torch.no_grad():
        for p, q in zip(P, Q):
            assert p.shape == q.shape, (p.shape, q.shape)
            q.copy_(p.float())
    g = torch.Generator().manual_seed(0)
    xs = [torch.randn(a.batch, *shape, generator=g) for _ in range(4)]
    ys = [torch.randint(0, nc, (a.batch,), generator=g) for _ in range(4)]
    xd = [x.to(dev, torch.bfloat16).float().contiguous(memory_format=torch.channels_last) for x in xs]
    yd = [y.to(dev) for y in ys]

    # one-step gradients: ours (native bf16) / stock autocast bf16 / stock fp32 (reference)
    x0, y0 = w.prepare(xs[0], ys[0])
    loss_ours, _ = w.train_step(x0, y0)
    go = [p.grad.detach().float().clone() for p in P]
    ref.zero_grad()
    F.cross_entropy(ref(xd[0]), yd[0]).backward()
    g32 = [q.grad.detach().clone() for q in Q]
    ref.zero_grad()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        lb = F.cross_entropy(ref(xd[0]), yd[0])
    lb.backward()
    g16 = [q.grad.detach().clone() for q in Q]
    names = [n for n, _ in w.model.named_parameters()]
    print(f"loss ours {float(loss_ours.detach()):.5f}  stock-bf16 {float(lb.detach()):.5f}")
    print(f"{'param':<40}{'ours vs fp32':>14}{'stock-bf16 vs fp32':>20}")
    worst = 0.0
    for n, a_, b_, c_ in zip(names, go, g16, g32):
        e1, e2 = rel(a_, c_), rel(b_, c_)
        worst = max(worst, e1 / max(e2, 1e-3))
        print(f"{n:<40}{e1:>14.4f}{e2:>20.4f}")
    print(f"worst ratio (ours err / stock-bf16 err): {worst:.2f}")

    # trajectory: plain SGD, same init, same batches
    w2 = mk(a.lr)
    zero_res(w2)
    with torch.no_grad():
        for p, q in zip(w2.model.parameters(), ref.parameters()):
            q.copy_(p.float())
    opt = torch.optim.SGD(ref.parameters(), lr=a.lr)
    lo, ls = [], []
    for i in range(a.steps):
        x, y = w2.prepare(xs[i % 4], ys[i % 4])
        l1, _ = w2.train_step(x, y)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            l2 = F.cross_entropy(ref(xd[i % 4]), yd[i % 4])
        opt.zero_grad()
        l2.backward()
        opt.step()
        lo.append(float(l1))
        ls.append(float(l2.detach()))
    print("step  ours    stock")
    for i in range(0, a.steps, max(a.steps // 10, 1)):
        print(f"{i:4d}  {lo[i]:.4f}  {ls[i]:.4f}")
    print(f"final {lo[-1]:.4f}  {ls[-1]:.4f}")


if __name__ == "__main__":
    main()
