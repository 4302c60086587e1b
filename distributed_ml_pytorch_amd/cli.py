"""Command-line front end; flag-compatible with /root/reference/example/main.py:140-155.

Reference flags (same names, defaults and meaning): --batch-size 64,
--test-batch-size 10000, --epochs 20, --lr 0.008, --num-pull 10, --num-push 10,
--cuda, --log-interval 100, --no-distributed, --rank, --world-size 3, --server,
--master localhost, --port 29500.  Rank 0 is the parameter server in the
central topology (reference roles, Makefile:13-20).

Additional flags select the model, data, parallel mode, PS topology,
staleness bound, precision, checkpointing and resume.
"""
from __future__ import annotations

import argparse
import json
import logging
import sys

from .runtime.dist import init_distributed, shutdown
from .runtime.trainer import TrainConfig, run_training


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Distbelief training example (MI355X-native)")
    # ---- reference flags ------------------------------------------------------
    p.add_argument("--batch-size", type=int, default=64, metavar="N")
    p.add_argument("--test-batch-size", type=int, default=10000, metavar="N")
    p.add_argument("--epochs", type=int, default=20, metavar="N")
    p.add_argument("--lr", type=float, default=0.008, metavar="LR")
    p.add_argument("--num-pull", type=int, default=10, metavar="N")
    p.add_argument("--num-push", type=int, default=10, metavar="N")
    p.add_argument("--cuda", action="store_true", default=False)
    p.add_argument("--log-interval", type=int, default=100, metavar="N")
    p.add_argument("--no-distributed", action="store_true", default=False)
    p.add_argument("--rank", type=int, default=None, metavar="N")
    p.add_argument("--world-size", type=int, default=3, metavar="N")
    p.add_argument("--server", action="store_true", default=False)
    p.add_argument("--master", type=str, default="localhost")
    p.add_argument("--port", type=str, default="29500")
    # ---- extensions -----------------------------------------------------------
    p.add_argument("--model", default="alexnet",
                   help="mlp | lenet | alexnet | resnet18 | resnet34 | resnet50 | vit_b16 ...")
    p.add_argument("--num-classes", type=int, default=None)
    p.add_argument("--dataset", default="synthetic", help="synthetic | cifar10 | mnist")
    p.add_argument("--data-dir", default="./data")
    p.add_argument("--n-train", type=int, default=50000)
    p.add_argument("--n-test", type=int, default=10000)
    p.add_argument("--mode", default="asgd", choices=["asgd", "sync", "single"])
    p.add_argument("--ps", default="central", choices=["central", "sharded", "sharded_async", "local"])
    p.add_argument("--payload", default="auto", choices=["auto", "gloo", "rccl"])
    p.add_argument("--backend", default="auto", choices=["auto", "gloo", "nccl"])
    p.add_argument("--staleness", type=int, default=1)
    p.add_argument("--pull-mode", default="overwrite", choices=["overwrite", "rebase"])
    p.add_argument("--wire-dtype", default="fp32", choices=["fp32", "bf16"])
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--momentum", type=float, default=0.0)
    p.add_argument("--weight-decay", type=float, default=0.0)
    p.add_argument("--lr-schedule", default="constant", choices=["constant", "inv_epoch"])
    p.add_argument("--max-steps", type=int, default=None)
    p.add_argument("--bucket-mb", type=float, default=0.0,
                   help="sync-DP all-reduce bucket (MB); 0 = measured on the group at start-up")
    p.add_argument("--label-smoothing", type=float, default=0.0)
    p.add_argument("--no-divergence-check", action="store_true", default=False,
                   help="keep training when the parameters go non-finite (the reference's "
                        "behaviour); default: halt with an error at the next log interval")
    p.add_argument("--deterministic", action="store_true", default=False,
                   help="bitwise-reproducible debugging mode (e.g. for asgd-vs-sync "
                        "differences): fp32 compute on PyTorch's deterministic kernels, no "
                        "atomics-based split reductions (see runtime/determinism.py)")
    p.add_argument("--checkpoint", default=None)
    p.add_argument("--checkpoint-every", type=int, default=0)
    p.add_argument("--resume", default=None,
                   help="checkpoint base: workers load <base>.worker<rank>.pt, the PS <base>")
    p.add_argument("--ps-resume", default=None, help="explicit parameter-server checkpoint")
    p.add_argument("--delta-scale", default="sum",
                   help="sharded PS: combine simultaneous pushes by 'sum' (Downpour), 'mean' or x")
    p.add_argument("--ps-worker-timeout", type=float, default=0.0,
                   help="central PS drops a worker silent for this many seconds (0 = never)")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--log-dir", default="log")
    p.add_argument("--no-eval", action="store_true", default=False)
    p.add_argument("--json", action="store_true", help="print the result dict as JSON")
    p.add_argument("-v", "--verbose", action="store_true")
    return p


def config_from_args(a) -> TrainConfig:
    mode = "single" if a.no_distributed else a.mode
    return TrainConfig(
        model=a.model, num_classes=a.num_classes, dataset=a.dataset, data_dir=a.data_dir,
        n_train=a.n_train, n_test=a.n_test, batch_size=a.batch_size,
        test_batch_size=a.test_batch_size, epochs=a.epochs, max_steps=a.max_steps, lr=a.lr,
        momentum=a.momentum, weight_decay=a.weight_decay, lr_schedule=a.lr_schedule,
        n_push=a.num_push, n_pull=a.num_pull, staleness=a.staleness, pull_mode=a.pull_mode,
        wire_dtype=a.wire_dtype, mode=mode, ps=a.ps, payload=a.payload, dtype=a.dtype,
        cuda=a.cuda, log_interval=a.log_interval, evaluate=not a.no_eval, seed=a.seed,
        log_dir=a.log_dir, checkpoint=a.checkpoint, checkpoint_every=a.checkpoint_every,
        resume=a.resume, ps_resume=a.ps_resume, delta_scale=a.delta_scale,
        ps_worker_timeout=a.ps_worker_timeout, bucket_mb=a.bucket_mb,
        label_smoothing=a.label_smoothing, divergence_check=not a.no_divergence_check,
        deterministic=a.deterministic)


def main(argv=None):
    a = build_parser().parse_args(argv)
    if a.verbose:
        logging.basicConfig(level=logging.INFO)
    print(a, flush=True)
    cfg = config_from_args(a)
    if a.no_distributed:
        info = init_distributed(0, 1, use_cuda=a.cuda)
    else:
        if a.rank is None:
            import os

            if "RANK" not in os.environ:
                raise SystemExit("--rank is required for distributed runs (or set RANK); "
                                 "use --no-distributed for single-process SGD")
        backend = a.backend
        if backend == "auto":
            backend = "nccl" if a.cuda else "gloo"
        info = init_distributed(a.rank, a.world_size, backend=backend,
                                master="127.0.0.1" if a.master == "localhost" else a.master,
                                port=a.port, use_cuda=a.cuda)
        if a.server and info.rank != 0:
            raise SystemExit("--server is rank 0 in the central topology")
    try:
        res = run_training(cfg, info)
    finally:
        shutdown()
    if a.json:
        print(json.dumps(res, default=str), flush=True)
    return res


if __name__ == "__main__":
    main(sys.argv[1:])
