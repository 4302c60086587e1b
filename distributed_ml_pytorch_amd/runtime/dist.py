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
import socket
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


# Hardware queues per process for every multi-rank GPU process.  Each rank runs
# several HIP streams at once (compute, the push/pull side stream, the wgrad
# side stream, one link stream per peer on a PS, and RCCL's internal streams);
# HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues (default 4) and
# streams that share a queue run back to back (profiles/links_stream_creation_r4.txt,
# profiles/hw_queue_policy_r5.txt).  The harness refuses values above 32.
MULTI_RANK_HW_QUEUES = 16


def apply_hw_queue_policy(world_size: int, env: dict | None = None) -> str | None:
    """Set ``GPU_MAX_HW_QUEUES`` for a multi-rank job (HIP reads it once, at its
    initialisation: call before the first ``torch.cuda`` call of the process, or
    on a child's environment).  An explicit setting wins.  Returns the value."""
    env = os.environ if env is None else env
    if world_size > 1:
        env.setdefault("GPU_MAX_HW_QUEUES", str(MULTI_RANK_HW_QUEUES))
    return env.get("GPU_MAX_HW_QUEUES")


def init_distributed(rank: int | None = None, world_size: int | None = None,
                     backend: str = "auto", master: str | None = None, port: str | None = None,
                     use_cuda: bool | None = None, timeout_s: float = 1800.0) -> DistInfo:
    rank = int(_env("RANK", rank if rank is not None else 0))
    world_size = int(_env("WORLD_SIZE", world_size if world_size is not None else 1))
    local_rank = int(_env("LOCAL_RANK", rank if world_size > 1 else 0))
    if use_cuda is None:
        use_cuda = torch.cuda.is_available()
    # DMP_DIST_BACKEND=gloo rehearses the multi-rank GPU path with several ranks
    # on one device (RCCL refuses two ranks per GPU)
    backend = _env("DMP_DIST_BACKEND", backend)
    if backend == "auto":
        backend = "nccl" if use_cuda else "gloo"
    device = torch.device("cpu")
    if use_cuda:
        n = torch.cuda.device_count()
        dev_idx = assign_device(local_rank, n, backend if world_size > 1 else "none",
                                int(_env("LOCAL_WORLD_SIZE", 0) or 0))
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
    if not dist.is_initialized():
        dist.init_process_group(backend, rank=rank, world_size=world_size,
                                timeout=datetime.timedelta(seconds=timeout_s))
    return DistInfo(rank, world_size, local_rank, backend, device)


class PreflightError(RuntimeError):
    """A multi-rank launch that cannot work (too few devices, two ranks on one
    GPU, an unreachable pair communicator, a collective that saw fewer ranks)."""


def assign_device(local_rank: int, device_count: int, backend: str, local_world: int = 0) -> int:
    """GPU index of this rank: ``cuda:LOCAL_RANK``, checked.

    With RCCL every rank must own a distinct device -- a launch with more local
    ranks than GPUs would otherwise wrap two ranks onto one GPU (the old
    ``local_rank % device_count``) and fail only at the first collective.  The
    gloo rehearsal backend may share a device explicitly (several ranks on the
    one GPU of a test box)."""
    if device_count < 1:
        raise PreflightError("no GPU visible to this rank")
    if backend == "nccl":
        if local_world and local_world > device_count:
            raise PreflightError(
                f"{local_world} local ranks but only {device_count} visible GPU(s): RCCL needs "
                "one GPU per rank (launch fewer ranks, or DMP_DIST_BACKEND=gloo to rehearse)")
        if local_rank >= device_count:
            raise PreflightError(f"local rank {local_rank} has no GPU of its own "
                                 f"({device_count} visible)")
        return local_rank
    return local_rank % device_count


def device_identity(device: torch.device) -> str:
    """Host-unique name of a device: ``host/uuid`` for a GPU (the PCI location
    when the runtime reports no UUID), ``host/cpu`` otherwise."""
    host = socket.gethostname()
    if device.type != "cuda":
        return f"{host}/cpu"
    p = torch.cuda.get_device_properties(device)
    uid = str(getattr(p, "uuid", "") or "")
    if not uid or uid.strip("0-") == "":
        uid = "pci:{:04x}:{:02x}:{:02x}".format(getattr(p, "pci_domain_id", 0),
                                                 getattr(p, "pci_bus_id", 0),
                                                 getattr(p, "pci_device_id", 0))
    return f"{host}/{uid}"


def check_distinct_devices(idents: list[str]) -> None:
    """Raise if two ranks report the same device."""
    seen: dict[str, int] = {}
    for r, d in enumerate(idents):
        if d in seen:
            raise PreflightError(f"ranks {seen[d]} and {r} both run on {d}: RCCL needs one "
                                 "GPU per rank")
        seen[d] = r


def preflight(info: DistInfo, host_group=None, pair_groups: dict | None = None,
              ps_rank: int = 0) -> dict:
    """Start-up checks of a multi-rank job, every rank calls it (the result is an
    OBSERVATION for the benchmark record, not a restatement of the config):

    1. all-reduce a ones tensor over the default group (RCCL on GPUs): the sum is
       the number of ranks the collective actually reached (``rccl_ranks``);
    2. all-gather every rank's device identity over the host group and, on RCCL,
       require them to be distinct;
    3. central topology (``pair_groups`` = {worker: 2-rank group}): ping every
       (PS, worker) pair communicator -- the PS sends ``worker`` to each worker,
       the worker answers ``-worker``; both check the value.

    Any mismatch raises :class:`PreflightError` (the launcher exits non-zero).
    Reference analogue: the 2-rank send/recv demo /root/reference/pytorch_p2p_ex.py:7-23
    (here run as a check over the real payload communicators).
    """
    out = {"backend": info.backend, "world": info.world_size}
    if not info.is_distributed:
        out.update(rccl_ranks=0, ranks_observed=1, devices_distinct=True, pairs_pinged=0)
        return out
    nccl = info.backend == "nccl"
    dev = info.device if nccl else torch.device("cpu")
    one = torch.ones(1, dtype=torch.float32, device=dev)
    dist.all_reduce(one)
    seen = int(round(float(one.item())))
    if seen != info.world_size:
        raise PreflightError(f"all-reduce over the default group reached {seen} of "
                             f"{info.world_size} ranks")
    idents = [None] * info.world_size
    dist.all_gather_object(idents, device_identity(info.device), group=host_group)
    # CPU ranks share "the host": distinctness is a GPU property (None on CPU)
    distinct = len(set(idents)) == len(idents) if info.device.type == "cuda" else None
    if nccl:
        check_distinct_devices(idents)
    pinged = 0
    if pair_groups:
        pdev = info.device if nccl else torch.device("cpu")
        if info.rank == ps_rank:
            for w in sorted(pair_groups):
                t = torch.full((1,), float(w), device=pdev)
                dist.send(t, w, group=pair_groups[w])
                dist.recv(t, w, group=pair_groups[w])
                if int(round(float(t.item()))) != -w:
                    raise PreflightError(f"pair ping PS<->{w}: got {float(t.item())}, want {-w}")
                pinged += 1
        elif info.rank in pair_groups:
            g = pair_groups[info.rank]
            t = torch.zeros(1, device=pdev)
            dist.recv(t, ps_rank, group=g)
            if int(round(float(t.item()))) != info.rank:
                raise PreflightError(f"pair ping from PS: got {float(t.item())}, "
                                     f"want {info.rank}")
            t.neg_()
            dist.send(t, ps_rank, group=g)
            pinged = 1
    out.update(rccl_ranks=seen if nccl else 0, ranks_observed=seen, devices_distinct=distinct,
               pairs_pinged=pinged, devices=idents)
    return out


def barrier(info: DistInfo):
    if info.is_distributed and dist.is_initialized():
        if info.backend == "nccl":
            dist.barrier(device_ids=[info.device.index])
        else:
            dist.barrier()


def shutdown():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
