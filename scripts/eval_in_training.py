"""Time Worker.evaluate() between hipGraph training steps (the bench's held-out
evaluation), ResNet-18 bs512, 8 held-out batches: per-call wall time."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
os.environ.setdefault("DMP_CONV_TUNE_SEED", os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "..", "tuning", "mi355x_tune_cache.json"))

import torch  # noqa: E402

from distributed_ml_pytorch_amd.runtime.dist import DistInfo  # noqa: E402
from distributed_ml_pytorch_amd.runtime.trainer import TrainConfig, Worker  # noqa: E402
from distributed_ml_pytorch_amd.utils.data import ttl_pools  # noqa: E402


def main():
    n_eval = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    info = DistInfo(device=torch.device("cuda", 0))
    cfg = TrainConfig(model="resnet18", batch_size=512, mode="asgd", ps="local", lr=0.05,
                      evaluate=False, verbose=False)
    w = Worker(cfg, info)
    w.enable_graph(True)
    tr, he = ttl_pools(512, w.input_shape, w.num_classes, w.device, 8, 8,
                       dtype=w.compute_dtype)
    for _ in range(20):
        w.train_step(*tr.next())
    torch.cuda.synchronize()
    for k in range(n_eval):
        t0 = time.perf_counter()
        loss, acc = w.evaluate(zip(he.x, he.y))
        t1 = time.perf_counter()
        for _ in range(5):
            w.train_step(*tr.next())
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"eval {k}: {1e3 * (t1 - t0):.2f} ms (loss {loss:.4f} acc {acc:.4f}); "
              f"5 train steps after it {1e3 * (t2 - t1):.2f} ms", flush=True)
    w.finish()


if __name__ == "__main__":
    main()
