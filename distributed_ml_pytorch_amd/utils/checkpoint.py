"""Checkpoint / resume (absent in the reference).

The PS shard is the single source of truth in Downpour SGD, so the server
checkpoints ``{flat fp32 params, version, stats}``; a worker checkpoint adds
its step counter, push accumulator, momentum and model buffers (BN running
statistics are not part of the pushed vector, as in the reference's ravel).

Files are written atomically (tmp + rename) and loaded with
``torch.load(weights_only=True)``: nothing in a checkpoint is executed.
"""
from __future__ import annotations

import os

import torch


def _atomic_save(obj, path: str):
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def save_ps_checkpoint(path: str, flat: torch.Tensor, version: int, stats: dict | None = None):
    counts = (stats or {}).get("counts", {})
    _atomic_save({"kind": "ps", "params": flat.detach().cpu().contiguous(), "version": int(version),
                  "counts": {str(k): int(v) for k, v in counts.items()}}, path)


def load_ps_checkpoint(path: str):
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if sd.get("kind") != "ps":
        raise ValueError(f"{path} is not a parameter-server checkpoint")
    return sd["params"], int(sd["version"]), sd.get("counts", {})


def save_worker_checkpoint(path: str, model: torch.nn.Module, optimizer=None, step: int = 0,
                           extra: dict | None = None):
    sd = {"kind": "worker", "step": int(step),
          "model": {k: v.detach().cpu() for k, v in model.state_dict().items()}}
    if optimizer is not None:
        acc = getattr(optimizer, "acc", None)
        mom = getattr(optimizer, "mom", None)
        sd["opt"] = {
            "idx": int(getattr(optimizer, "idx", step)),
            "lr": float(optimizer.param_groups[0]["lr"]),
            "acc": acc.detach().cpu() if acc is not None else None,
            "mom": mom.detach().cpu() if mom is not None else None,
        }
        client = getattr(optimizer, "client", None)
        if client is not None:
            # PS state held on this worker (in-process master / its sharded-PS shard)
            sd["client"] = client.state_dict()
    if extra:
        sd["extra"] = extra
    _atomic_save(sd, path)


def _load_worker_sd(path: str) -> dict:
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if sd.get("kind") != "worker":
        raise ValueError(f"{path} is not a worker checkpoint")
    return sd


def load_worker_model(path: str, model: torch.nn.Module) -> int:
    """Restore model parameters/buffers (into the arena views) and return the step.

    Call BEFORE the optimizer is built: the PS client seeds its master (or the
    central PS) from the live parameters in ``client.init()``.
    """
    sd = _load_worker_sd(path)
    with torch.no_grad():
        own = model.state_dict()
        for k, v in sd["model"].items():
            own[k].copy_(v)
    from ..parallel.arena import get_arena

    arena = get_arena(model)
    if arena is not None:
        arena.refresh_shadow()
        arena.bump()
    return int(sd["step"])


def load_worker_optimizer(path: str, optimizer) -> None:
    """Restore the optimizer (step index, lr, push accumulator, momentum) and the
    PS state its client holds (local master, sharded-PS shard)."""
    sd = _load_worker_sd(path)
    if "opt" in sd:
        o = sd["opt"]
        if hasattr(optimizer, "idx"):
            optimizer.idx = o["idx"]
        for g in optimizer.param_groups:
            g["lr"] = o["lr"]
        with torch.no_grad():
            if o.get("acc") is not None and getattr(optimizer, "acc", None) is not None:
                optimizer.acc.copy_(o["acc"])
            if o.get("mom") is not None and getattr(optimizer, "mom", None) is not None:
                optimizer.mom.copy_(o["mom"])
                optimizer._mom_steps = max(1, int(o.get("idx", 1)))   # buffer already seeded
    client = getattr(optimizer, "client", None)
    if client is not None and sd.get("client"):
        client.load_state_dict(sd["client"])


def load_worker_checkpoint(path: str, model: torch.nn.Module, optimizer=None) -> int:
    step = load_worker_model(path, model)
    if optimizer is not None:
        load_worker_optimizer(path, optimizer)
    return step


def worker_checkpoint_path(base: str, rank: int) -> str:
    """Per-rank worker file derived from one ``--checkpoint``/``--resume`` base
    (the PS writes ``base`` itself)."""
    root, ext = os.path.splitext(base)
    return f"{root}.worker{rank}{ext or '.pt'}"


def checkpoint_kind(path: str) -> str | None:
    try:
        return torch.load(path, map_location="cpu", weights_only=True).get("kind")
    except (FileNotFoundError, RuntimeError, ValueError):
        return None
