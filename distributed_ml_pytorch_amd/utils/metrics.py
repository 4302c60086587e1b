"""Per-iteration training log + throughput meters (reference §5.5).

The reference appends ``{timestamp, iteration, training_loss[, test_loss,
test_accuracy]}`` per iteration and writes a pandas CSV to
``log/{single,gpu,node<rank>}.csv`` (/root/reference/example/main.py:76-105),
crashing when ``log/`` does not exist.  Same schema here, plus
``epoch``, ``samples_per_sec`` and free-form extras; the directory is created.
GPU losses are accumulated as tensors and only synchronised at log points,
so logging never stalls the step pipeline (the reference synced every step
with ``loss.item()``, main.py:79).
"""
from __future__ import annotations

import csv
import os
import time
from datetime import datetime

import torch

BASE_FIELDS = ["index", "timestamp", "epoch", "iteration", "training_loss", "test_loss",
               "test_accuracy", "samples_per_sec"]


class IterationLog:
    def __init__(self):
        self.rows: list[dict] = []
        self._pending: list[tuple[dict, torch.Tensor]] = []

    def append(self, epoch: int, iteration: int, loss, **extra):
        row = {"timestamp": datetime.now().isoformat(sep=" "), "epoch": epoch,
               "iteration": iteration, **extra}
        if isinstance(loss, torch.Tensor):
            self._pending.append((row, loss.detach()))
        else:
            row["training_loss"] = float(loss)
        self.rows.append(row)
        return row

    def flush_pending(self):
        if not self._pending:
            return
        vals = torch.stack([t.float().reshape(()) for _, t in self._pending]).tolist()
        for (row, _), v in zip(self._pending, vals):
            row["training_loss"] = v
        self._pending.clear()

    def last(self) -> dict:
        self.flush_pending()
        return self.rows[-1] if self.rows else {}

    def to_csv(self, path: str):
        self.flush_pending()
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        fields = list(BASE_FIELDS)
        for r in self.rows:
            for k in r:
                if k not in fields:
                    fields.append(k)
        with open(path, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=fields)
            w.writeheader()
            for i, r in enumerate(self.rows):
                w.writerow({"index": i, **r})
        return path


def log_path(no_distributed: bool, cuda: bool, rank: int | None, log_dir: str = "log") -> str:
    if no_distributed:
        return os.path.join(log_dir, "gpu.csv" if cuda else "single.csv")
    return os.path.join(log_dir, f"node{rank}.csv")


class Throughput:
    """Wall-clock samples/sec with optional device synchronisation."""

    def __init__(self, sync_cuda: bool = False):
        self.sync_cuda = sync_cuda
        self.reset()

    def reset(self):
        if self.sync_cuda:
            torch.cuda.synchronize()
        self.t0 = time.perf_counter()
        self.samples = 0

    def add(self, n: int):
        self.samples += n

    def rate(self) -> float:
        if self.sync_cuda:
            torch.cuda.synchronize()
        dt = time.perf_counter() - self.t0
        return self.samples / dt if dt > 0 else 0.0


class StepTimer:
    """Accumulates named host-side phase times (compute, push, pull-wait, ...)."""

    def __init__(self):
        self.totals: dict[str, float] = {}
        self.counts: dict[str, int] = {}

    def time(self, name: str):
        timer = self

        class _Ctx:
            def __enter__(self_inner):
                self_inner.t = time.perf_counter()

            def __exit__(self_inner, *a):
                dt = time.perf_counter() - self_inner.t
                timer.totals[name] = timer.totals.get(name, 0.0) + dt
                timer.counts[name] = timer.counts.get(name, 0) + 1
                return False

        return _Ctx()

    def summary(self) -> dict:
        return {k: {"total_s": v, "mean_ms": 1e3 * v / max(self.counts[k], 1)}
                for k, v in self.totals.items()}
