"""Which CPU op launched each non-native device kernel of one training step (torch
profiler, with Python stacks).  python scripts/find_stock_kernels.py --model resnet50 --batch 4"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from distributed_ml_pytorch_amd.runtime.dist import DistInfo  # noqa: E402
from distributed_ml_pytorch_amd.runtime.trainer import TrainConfig, Worker  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=4)
    a = ap.parse_args()
    w = Worker(TrainConfig(model=a.model, batch_size=a.batch, mode="asgd", ps="local", n_push=1,
                           n_pull=1, lr=0.01, evaluate=False, verbose=False),
               DistInfo(device=torch.device("cuda", 0)))
    x = torch.randn(a.batch, *w.input_shape)
    y = torch.randint(0, w.num_classes, (a.batch,))
    x, y = w.prepare(x, y)
    w.train_step(x, y)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        w.train_step(x, y)
        torch.cuda.synchronize()
    seen = 0
    for e in prof.events():
        for k in getattr(e, "kernels", []):
            if "dmp::" in k.name or k.name.startswith(("__amd_rocclr_copyBuffer", "Memcpy")):
                continue
            seen += 1
            print(f"== {k.name}  <-  {e.name}")
            for fr in (e.stack or [])[:12]:
                print("     ", fr)
    print(f"{seen} non-native kernel launch(es)")


if __name__ == "__main__":
    main()
