"""Virtual workers: the reference's 1 PS + N workers ASGD topology inside ONE process.

The reference runs Downpour SGD as separate processes - rank 0 the parameter
server, ranks 1..N workers (``Makefile:13-20``, ``example/main.py:151-168``).
RCCL refuses two ranks on one GPU, so on a single MI355X the multi-worker
asynchrony is reproduced here instead: K full model replicas
share one device, each steps on its own HIP stream (kernels of different
workers overlap on the CUs), and all of them push to / pull from one
:class:`~..parallel.clients.SharedPS` whose applies are serialised on the PS
stream.  Each worker keeps the reference cadence (push every ``n_push``, pull
every ``n_pull``, ``Asynchronous.py:48-70``) and its own data order (no
DistributedSampler, ``main.py:27``).
"""
from __future__ import annotations

import contextlib
from dataclasses import replace

import torch

from ..parallel.clients import SharedPS, SharedPSClient
from .dist import DistInfo
from .trainer import TrainConfig, Worker, _dtype


class VirtualWorkers:
    def __init__(self, cfg: TrainConfig, k: int, device: torch.device | None = None):
        if k < 1:
            raise ValueError("need at least one virtual worker")
        if cfg.mode != "asgd":
            raise ValueError("virtual workers run the asynchronous (asgd) mode")
        device = device or (torch.device("cuda", 0) if torch.cuda.is_available() and cfg.cuda
                            else torch.device("cpu"))
        self.device = device
        self.cuda = device.type == "cuda"
        self.shared = SharedPS()
        self.workers: list[Worker] = []
        self.streams = [torch.cuda.Stream(device) if self.cuda else None for _ in range(k)]
        kw = dict(staleness=cfg.staleness, pull_mode=cfg.pull_mode,
                  wire_dtype=_dtype(cfg.wire_dtype))
        for i in range(k):
            with self._on(i):
                w = Worker(replace(cfg, seed=cfg.seed + i), DistInfo(device=device),
                           client=SharedPSClient(self.shared, **kw))
            self.workers.append(w)

    def _on(self, i: int):
        return torch.cuda.stream(self.streams[i]) if self.cuda else contextlib.nullcontext()

    def enable_graph(self, enabled: bool = True) -> bool:
        return all([w.enable_graph(enabled) for w in self.workers]) if self.cuda else False

    def step(self, batches):
        """One step of every worker on its own stream; ``batches[i] = (x, y)``.
        Returns the per-worker losses (device tensors, no host sync)."""
        losses = []
        for i, (w, (x, y)) in enumerate(zip(self.workers, batches)):
            with self._on(i):
                loss, _ = w.train_step(x, y)
            losses.append(loss)
        return losses

    def master(self) -> torch.Tensor:
        """The PS parameters after every enqueued push (waits on the PS stream)."""
        if self.shared.stream is not None:
            torch.cuda.current_stream().wait_stream(self.shared.stream)
        return self.shared.master

    def finish(self):
        for i, w in enumerate(self.workers):
            with self._on(i):
                w.finish()
        if self.cuda:
            for s in self.streams:
                torch.cuda.current_stream().wait_stream(s)
            if self.shared.stream is not None:
                torch.cuda.current_stream().wait_stream(self.shared.stream)

    def stats(self) -> list[dict]:
        return [w.opt.stats() for w in self.workers]
