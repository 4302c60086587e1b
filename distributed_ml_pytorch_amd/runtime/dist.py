"""Process-group bootstrap: one process per GPU, RCCL (``nccl``) on GPUs, gloo on CPU.

Replaces the reference's hard-coded ``init_process_group('gloo', rank,
world_size)`` (/root/reference/example/main.py:163-165, pytorch_p2p_ex.py:20-22)
with env:// rendezvous that works under ``torch.distributed.run`` (RANK /
WORLD_SIZE / LOCAL_RANK / MASTER_*), the repo's own launcher, or explicit
``--rank/--world-size`` flags, and binds each rank to ``cuda:LOCAL_RANK``.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1


def _env(name, default=None):
    v = os.environ.get(name)
    return default if v is None or v == "" else v


def init_distributed(rank: int | None = None, world_size: int | None = None,
                     backend: str = "auto", master: str | None = None, port: str | None = None,
                     use_cuda: bool | None = None, timeout_s: float = 1800.0) -> DistInfo:
    rank = int(_env("RANK", rank if rank is not None else 0))
    world_size = int(_env("WORLD_SIZE", world_size if world_size is not None else 1))
    local_rank = int(_env("LOCAL_RANK", rank if world_size > 1 else 0))
    if use_cuda is None:
        use_cuda = torch.cuda.is_available()
    device = torch.device("cpu")
    if use_cuda:
        n = torch.cuda.device_count()
        dev_idx = local_rank % max(n, 1)
        torch.cuda.set_device(dev_idx)
        device = torch.device("cuda", dev_idx)
    if world_size <= 1:
        return DistInfo(0, 1, 0, "none", device)
    os.environ.setdefault("MASTER_ADDR", master or "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(port or 29500))
    if master:
        os.environ["MASTER_ADDR"] = master
    if port:
        os.environ["MASTER_PORT"] = str(port)
    # DMP_DIST_BACKEND=gloo rehearses the multi-rank GPU path with several ranks
    # on one device (RCCL refuses two ranks per GPU)
    backend = _env("DMP_DIST_BACKEND", backend)
    if backend == "auto":
        backend = "nccl" if use_cuda else "gloo"
    if not dist.is_initialized():
        dist.init_process_group(backend, rank=rank, world_size=world_size,
                                timeout=datetime.timedelta(seconds=timeout_s))
    return DistInfo(rank, world_size, local_rank, backend, device)


def barrier(info: DistInfo):
    if info.is_distributed and dist.is_initialized():
        if info.backend == "nccl":
            dist.barrier(device_ids=[info.device.index])
        else:
            dist.barrier()


def shutdown():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
