"""Stock PyTorch-ROCm comparison point for the bench configs (BASELINE.md
"comparison point": stock PyTorch-ROCm runs of the same configs on the same
MI355X).

Same architectures as ``distributed_ml_pytorch_amd.models`` (ResNet-18 CIFAR
stem, ResNet-50 ImageNet stem, ViT-B/16 224^2) written with plain ``torch.nn``
modules only: MIOpen convolutions / BatchNorm, hipBLASLt linears, ATen SDPA,
``torch.autocast(bfloat16)`` over fp32 master weights, channels-last,
``torch.optim.SGD(fused=True)``.  Synthetic HBM-resident batches, random init.
The timed region is forward + backward + optimizer step, like ``bench.py``.

``--graph`` (round 6, VERDICT r5 #8: a fair comparator): the same step captured
once into a ``torch.cuda.CUDAGraph`` (static input / label buffers refilled by a
device copy each step, as bench.py's graph refills its own) and replayed, so the
stock arm pays no per-op host launch either -- what is left is kernel quality.

    python scripts/stock_baseline.py --model resnet18 --batch 256 --steps 30 [--graph]
"""
from __future__ import annotations

import argparse
import json
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class Basic(nn.Module):
    exp = 1

    def __init__(self, cin, planes, stride):
        super().__init__()
        self.c1 = nn.Conv2d(cin, planes, 3, stride, 1, bias=False)
        self.b1 = nn.BatchNorm2d(planes)
        self.c2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.b2 = nn.BatchNorm2d(planes)
        self.sc = None
        if stride != 1 or cin != planes:
            self.sc = nn.Sequential(nn.Conv2d(cin, planes, 1, stride, bias=False),
                                    nn.BatchNorm2d(planes))

    def forward(self, x):
        h = F.relu(self.b1(self.c1(x)))
        return F.relu(self.b2(self.c2(h)) + (x if self.sc is None else self.sc(x)))


class Bottle(nn.Module):
    exp = 4

    def __init__(self, cin, planes, stride):
        super().__init__()
        out = planes * 4
        self.c1 = nn.Conv2d(cin, planes, 1, bias=False)
        self.b1 = nn.BatchNorm2d(planes)
        self.c2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.b2 = nn.BatchNorm2d(planes)
        self.c3 = nn.Conv2d(planes, out, 1, bias=False)
        self.b3 = nn.BatchNorm2d(out)
        self.sc = None
        if stride != 1 or cin != out:
            self.sc = nn.Sequential(nn.Conv2d(cin, out, 1, stride, bias=False), nn.BatchNorm2d(out))

    def forward(self, x):
        h = F.relu(self.b1(self.c1(x)))
        h = F.relu(self.b2(self.c2(h)))
        return F.relu(self.b3(self.c3(h)) + (x if self.sc is None else self.sc(x)))


class ResNet(nn.Module):
    def __init__(self, block, layers, nc, imagenet):
        super().__init__()
        if imagenet:
            self.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64),
                                      nn.ReLU(inplace=True), nn.MaxPool2d(3, 2, 1))
        else:
            self.stem = nn.Sequential(nn.Conv2d(3, 64, 3, 1, 1, bias=False), nn.BatchNorm2d(64),
                                      nn.ReLU(inplace=True))
        blocks, cin = [], 64
        for i, n in enumerate(layers):
            planes = 64 << i
            for j in range(n):
                blocks.append(block(cin, planes, 2 if (j == 0 and i > 0) else 1))
                cin = planes * block.exp
        self.blocks = nn.Sequential(*blocks)
        self.fc = nn.Linear(cin, nc)

    def forward(self, x):
        h = self.blocks(self.stem(x))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(h, 1), 1))


class Block(nn.Module):
    def __init__(self, d, heads, mlp):
        super().__init__()
        self.h = heads
        self.ln1 = nn.LayerNorm(d, eps=1e-6)
        self.qkv = nn.Linear(d, 3 * d)
        self.proj = nn.Linear(d, d)
        self.ln2 = nn.LayerNorm(d, eps=1e-6)
        self.fc1 = nn.Linear(d, mlp)
        self.fc2 = nn.Linear(mlp, d)

    def forward(self, x):
        b, t, d = x.shape
        q, k, v = self.qkv(self.ln1(x)).view(b, t, 3, self.h, d // self.h).permute(2, 0, 3, 1, 4)
        a = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(b, t, d)
        x = x + self.proj(a)
        return x + self.fc2(F.gelu(self.fc1(self.ln2(x))))


class ViT(nn.Module):
    def __init__(self, nc=1000, img=224, patch=16, d=768, depth=12, heads=12, mlp=3072):
        super().__init__()
        self.patch = nn.Conv2d(3, d, patch, patch)
        n = (img // patch) ** 2
        self.cls = nn.Parameter(torch.zeros(1, 1, d))
        self.pos = nn.Parameter(torch.randn(1, n + 1, d) * 0.02)
        self.blocks = nn.Sequential(*[Block(d, heads, mlp) for _ in range(depth)])
        self.ln = nn.LayerNorm(d, eps=1e-6)
        self.head = nn.Linear(d, nc)

    def forward(self, x):
        h = self.patch(x).flatten(2).transpose(1, 2)
        h = torch.cat([self.cls.expand(h.shape[0], -1, -1), h], 1) + self.pos
        return self.head(self.ln(self.blocks(h))[:, 0])


MODELS = {
    "resnet18": (lambda: ResNet(Basic, [2, 2, 2, 2], 10, False), (3, 32, 32), 10),
    "resnet50": (lambda: ResNet(Bottle, [3, 4, 6, 3], 1000, True), (3, 224, 224), 1000),
    "vit_b16": (lambda: ViT(), (3, 224, 224), 1000),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18", choices=sorted(MODELS))
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--graph", action="store_true",
                    help="capture fwd + bwd + fused SGD in one CUDAGraph and replay it")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    ctor, shape, nc = MODELS[a.model]
    model = ctor().to(dev).to(memory_format=torch.channels_last)
    nparam = sum(p.numel() for p in model.parameters())
    opt = torch.optim.SGD(model.parameters(), lr=a.lr, fused=True)
    g = torch.Generator(device=dev).manual_seed(0)
    xs = [torch.randn(a.batch, *shape, device=dev, generator=g).to(memory_format=torch.channels_last)
          for _ in range(4)]
    ys = [torch.randint(0, nc, (a.batch,), device=dev, generator=g) for _ in range(4)]

    def step(i):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(model(xs[i % 4]), ys[i % 4])
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    if a.graph:
        sx, sy = xs[0].clone(), ys[0].clone()

        def body():
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = F.cross_entropy(model(sx), sy)
            loss.backward()
            opt.step()
            return loss

        # warm up on a side stream (MIOpen algorithm search, lazy allocations), then
        # capture with the gradients unset so their buffers come from the graph pool
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(3, a.warmup)):
                opt.zero_grad(set_to_none=True)
                body()
        torch.cuda.current_stream().wait_stream(side)
        opt.zero_grad(set_to_none=True)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            static_loss = body()

        def step(i):   # noqa: F811  (the graphed step: refill the inputs, replay)
            sx.copy_(xs[i % 4])
            sy.copy_(ys[i % 4])
            graph.replay()
            return static_loss

    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = step(i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    mode = "CUDAGraph-captured" if a.graph else "eager"
    print(json.dumps({"impl": f"stock-pytorch-rocm {mode} (autocast bf16, channels_last, MIOpen, "
                              "SDPA, fused SGD)", "torch": torch.__version__, "model": a.model,
                      "params": nparam, "batch": a.batch, "steps": a.steps,
                      "ms_per_step": round(1e3 * el / a.steps, 3),
                      "samples_per_s": round(a.batch * a.steps / el, 1),
                      "loss": round(float(loss.detach().float()), 4)}), flush=True)


if __name__ == "__main__":
    main()
