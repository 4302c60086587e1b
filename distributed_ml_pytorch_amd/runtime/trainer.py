"""Training driver: the reference's ``example/main.py`` loop as a reusable engine.

Roles and loop follow /root/reference/example/main.py:31-138 (rank 0 = PS in
the central topology, workers train with ``Asynchronous``; ``--no-distributed``
= plain SGD), plus the modes BASELINE.json asks for:

* ``mode="asgd"``   Downpour SGD; ``ps`` = ``central`` (reference star,
  gloo or RCCL payloads), ``sharded`` (PS co-located on every GPU, collective
  push/pull), ``sharded_async`` (one PS thread per shard, point-to-point
  push/pull, no rank waits for another: parallel/async_sharded.py) or
  ``local`` (in-process PS, 1 device);
* ``mode="sync"``   bucketed all-reduce data parallel;
* ``mode="single"`` plain SGD, no communication.

Per step: zero the flat grad arena (one memset) -> bf16 channels-last forward
through the native layers -> fused softmax-xent -> backward (native kernels
write fp32 weight grads straight into the arena) -> [bucket sync] -> fused
optimizer kernel (+ push/pull).  No host sync per step: the loss is kept on
device and only read at log points.
"""
from __future__ import annotations

import logging
import math
import os
import time
from dataclasses import asdict, dataclass, field

import torch
import torch.distributed as dist

from ..models import build_model
from ..ops.eval_fold import fold_session
from ..ops.functional import softmax_cross_entropy, unit_grad
from ..parallel.arena import attach_arena
from ..parallel.asgd import Asynchronous
from ..parallel.async_sharded import AsyncShardedPSClient
from ..parallel.clients import (GlooPSClient, LocalPSClient, RcclPSClient, ShardedPSClient)
from ..parallel.ddp import BucketedAllReduce, FusedSGD
from ..parallel.server import ParameterServer, make_ps_groups
from ..utils import checkpoint as ckpt
from ..utils.data import get_datasets, make_loaders
from ..utils.metrics import IterationLog, StepTimer, Throughput, classification_report
from .determinism import enable_determinism
from .dist import DistInfo, preflight

_LOG = logging.getLogger(__name__)


class DivergenceError(RuntimeError):
    """Training produced non-finite parameters (the log-interval watchdog)."""


@dataclass
class TrainConfig:
    model: str = "alexnet"
    num_classes: int | None = None
    dataset: str = "synthetic"
    data_dir: str = "./data"
    n_train: int = 50000
    n_test: int = 10000
    batch_size: int = 64
    test_batch_size: int = 10000
    epochs: int = 20
    max_steps: int | None = None
    lr: float = 0.008
    momentum: float = 0.0
    weight_decay: float = 0.0
    lr_schedule: str = "constant"     # or "inv_epoch": the reference's LambdaLR(1/(epoch+1))
    n_push: int = 10
    n_pull: int = 10
    staleness: int = 1
    pull_mode: str = "overwrite"
    wire_dtype: str = "fp32"
    mode: str = "asgd"                # asgd | sync | single
    ps: str = "central"               # central | sharded | sharded_async | local
    payload: str = "auto"             # central PS payload transport: gloo | rccl | auto
    dtype: str = "bf16"               # compute dtype on GPU (CPU always fp32)
    cuda: bool = True
    log_interval: int = 100
    evaluate: bool = True
    seed: int = 0
    log_dir: str = "log"
    checkpoint: str | None = None
    checkpoint_every: int = 0
    resume: str | None = None         # base path: workers read <base>.worker<rank>.pt, the PS <base>
    ps_resume: str | None = None      # explicit PS checkpoint (overrides <base> for the PS)
    delta_scale: str = "sum"          # PS push combine: "sum" (Downpour PS semantics) | "mean" | float
    ps_worker_timeout: float = 0.0    # central PS: drop a worker silent this long (0 = never)
    bucket_mb: float = 0.0            # sync-DP all-reduce bucket; <= 0: measured (ddp.py)
    label_smoothing: float = 0.0
    divergence_check: bool = True     # halt on non-finite parameters at each log interval
    deterministic: bool = False       # bitwise-reproducible debug mode (runtime/determinism.py)
    verbose: bool = True
    extra: dict = field(default_factory=dict)


def _dtype(name: str) -> torch.dtype:
    return {"bf16": torch.bfloat16, "bfloat16": torch.bfloat16, "fp32": torch.float32,
            "float32": torch.float32, "fp16": torch.float16}[name]


class Worker:
    """One training process: model + arena + optimizer + step function."""

    def __init__(self, cfg: TrainConfig, info: DistInfo, ps_groups=None, client=None):
        """``client``: an explicit PS client for ``mode='asgd'`` (e.g. a
        :class:`~..parallel.clients.SharedPSClient` of the virtual-worker runner)."""
        self.cfg = cfg
        self.info = info
        if cfg.deterministic:
            cfg = self.cfg = enable_determinism(cfg)
        torch.manual_seed(cfg.seed + info.rank)
        self.device = info.device if (cfg.cuda and info.device.type == "cuda") else \
            torch.device("cpu")
        self.compute_dtype = _dtype(cfg.dtype) if self.device.type == "cuda" else torch.float32
        if self.device.type == "cuda" and self.compute_dtype != torch.bfloat16:
            from ..ops._policy import is_allowed

            if not is_allowed():
                # the native kernels are bf16-compute (fp32 masters / accumulation);
                # an fp32 GPU run would train entirely on MIOpen / hipBLASLt / ATen
                raise ValueError(
                    f"--dtype {cfg.dtype} on the GPU: every native gfx950 kernel computes "
                    "in bf16 (fp32 master weights and accumulation), so this would train "
                    "entirely on stock MIOpen / hipBLASLt / ATen kernels.  Use --dtype bf16, "
                    "or --deterministic for the explicit fp32 stock-kernel oracle mode.")
        model, shape, nc = build_model(cfg.model, cfg.num_classes)
        self.input_shape, self.num_classes = shape, nc
        self.model = model.to(self.device)
        shadow = self.compute_dtype if self.compute_dtype != torch.float32 else None
        self.arena = attach_arena(self.model, shadow_dtype=shadow,
                                  channels_last=True)
        self.ddp = None
        self.timer = StepTimer()
        self.step_idx = 0
        # resume the parameters BEFORE the optimizer exists: its PS client seeds the
        # master (local / sharded) or the central PS from the live parameters
        resume = _worker_resume_path(cfg.resume, info.rank) if cfg.resume else None
        if cfg.resume and info.is_distributed and not (cfg.mode == "asgd" and cfg.ps == "central"):
            # every rank of a collective topology must take the same decision: the
            # sharded clients restore through a collective, so one rank starting
            # fresh while the others resume would hang them (central-PS workers
            # resume independently: a fresh one adopts the PS params at its pull)
            _agree_on_resume(resume is not None, info)
        if resume:
            self.step_idx = ckpt.load_worker_model(resume, self.model)
        params = list(self.model.parameters())
        if cfg.mode == "asgd":
            client = client if client is not None else self._make_client(ps_groups)
            self.opt = Asynchronous(params, lr=cfg.lr, n_push=cfg.n_push, n_pull=cfg.n_pull,
                                    model=self.model, client=client, momentum=cfg.momentum,
                                    weight_decay=cfg.weight_decay)
        elif cfg.mode == "sync":
            world = dist.get_world_size() if info.is_distributed else 1
            if info.is_distributed:
                dist.broadcast(self.arena.p32, 0)
                self.arena.refresh_shadow()
            self.ddp = BucketedAllReduce(self.arena, bucket_mb=cfg.bucket_mb)
            self.opt = FusedSGD(params, self.arena, cfg.lr, cfg.momentum,
                                weight_decay=cfg.weight_decay, grad_scale=1.0 / world)
        elif cfg.mode == "single":
            self.opt = FusedSGD(params, self.arena, cfg.lr, cfg.momentum,
                                weight_decay=cfg.weight_decay)
        else:
            raise ValueError(f"unknown mode {cfg.mode!r}")
        if isinstance(self.opt, Asynchronous):
            self.opt.timer = self.timer
        if resume:
            ckpt.load_worker_optimizer(resume, self.opt)

    def _make_client(self, ps_groups):
        cfg, info = self.cfg, self.info
        kw = dict(staleness=cfg.staleness, pull_mode=cfg.pull_mode,
                  wire_dtype=_dtype(cfg.wire_dtype))
        if cfg.ps == "local" or not info.is_distributed:
            return LocalPSClient(**kw)
        if cfg.ps == "sharded":
            return ShardedPSClient(delta_scale=cfg.delta_scale, **kw)
        if cfg.ps == "sharded_async":
            return AsyncShardedPSClient(delta_scale=cfg.delta_scale, **kw)
        if cfg.ps == "central":
            ctrl, pairs = ps_groups if ps_groups is not None else (None, {})
            if pairs and self.device.type == "cuda" and _payload(cfg, info) == "rccl":
                return RcclPSClient(0, ctrl, pairs[info.rank], **kw)
            return GlooPSClient(ps_rank=0, group=ctrl, **kw)
        raise ValueError(f"unknown ps kind {cfg.ps!r}")

    # --------------------------------------------------------------- stepping
    def prepare(self, x, y):
        x = x.to(self.device, non_blocking=True)
        if self.device.type == "cuda":
            x = x.to(self.compute_dtype)
            if x.dim() == 4:
                x = x.contiguous(memory_format=torch.channels_last)
        return x, y.to(self.device, non_blocking=True)

    # ------------------------------------------------------------ hipGraph path
    def enable_graph(self, enabled: bool = True):
        """Replay forward+backward+fused update as ONE captured hipGraph per step.

        The push/pull/land half of the ASGD step (which depends on the step
        index) stays eager between replays.  Sync DP is captured whole: the
        bucket all-reduces that the grad-ready hooks launch during backward
        (RCCL on the comm stream, ordered by events) and the wait before the
        update are part of the graph.  Gloo collectives cannot be captured:
        sync DP over gloo stays eager.
        """
        can = self.device.type == "cuda"
        if self.ddp is not None and self.info.is_distributed:
            # gloo collectives cannot be captured; RCCL ones can, OPT-IN
            # (DMP_GRAPH_SYNC=1): eager sync DP pays the host launch of every
            # dispatch (~350 per ResNet-50 step, profiles/sync_dp_capture_ab_r4.txt),
            # but that A/B ran at world 1 and a captured multi-rank all-reduce has
            # not been replayed on a multi-GPU node yet, so multi-rank sync DP
            # steps eagerly by default.  With capture on, a capture that fails on
            # ANY rank makes every rank step eagerly (_capture_agreed).
            can = can and self.info.backend == "nccl" and \
                os.environ.get("DMP_GRAPH_SYNC", "0") == "1"
        self.use_graph = bool(enabled) and can
        self.graph = None
        return self.use_graph

    def _graph_body(self):
        self.opt.zero_grad()
        logits = self.model(self._gx)
        loss, hits = softmax_cross_entropy(logits, self._gy, self.cfg.label_smoothing)
        loss.backward(unit_grad(loss))
        if self.ddp is not None:
            self.ddp.synchronize()
        self.opt.local_step()
        return loss.detach(), hits

    def _capture(self, x, y):
        """Run this step eagerly on a side stream (tunes kernels, warms the
        allocator and libraries), then capture the step body for later replays."""
        self._gx = x.detach().clone()
        self._gy = y.detach().clone()
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            loss, hits = self._graph_body()
            self.opt.comm_step()
            self.step_idx += 1
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        err = None
        try:
            # thread_local: RCCL's watchdog thread queries events while we capture
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                self._gloss, self._ghits = self._graph_body()
        except RuntimeError as e:     # e.g. a collective backend that cannot be captured
            err = str(e)
            if self.ddp is not None:
                self.ddp.reset()
        # sync DP: every rank replays or every rank steps eagerly -- a rank whose
        # capture failed must not run a different launch path from its peers
        # (capture records the collectives, it does not run them, so this
        # agreement all-reduce is the first collective after the eager step)
        if self.ddp is not None and self.info.is_distributed and \
                not self._capture_agreed(err is None):
            err = err or "a peer rank's capture failed"
            self.ddp.reset()
        if err is not None:
            print(f"[trainer] hipGraph capture failed ({err}); stepping eagerly", flush=True)
            self.use_graph = False
            self.graph = None
            return loss.clone(), hits.clone()
        self.graph = g
        self._graph_key = (tuple(x.shape), x.dtype, self.opt.param_groups[0]["lr"])
        return loss.clone(), hits.clone()

    def _capture_agreed(self, ok: bool) -> bool:
        """MIN-all-reduce of the local capture verdict over the sync-DP group."""
        import torch.distributed as dist

        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.ddp.group)
        return bool(flag.item())

    def _graph_step(self, x, y, keep: bool = True):
        key = (tuple(x.shape), x.dtype, self.opt.param_groups[0]["lr"])
        if self.graph is None or key != self._graph_key:
            return self._capture(x, y)
        with self.timer.time("compute_launch"):
            self._gx.copy_(x, non_blocking=True)
            self._gy.copy_(y, non_blocking=True)
            self.graph.replay()
        self.opt.comm_step()
        self.step_idx += 1
        # the captured outputs are overwritten by the next replay: copies unless
        # the caller reads them before the next step (``keep=False``)
        if not keep:
            return self._gloss, self._ghits
        return self._gloss.clone(), self._ghits.clone()

    def param_norm(self) -> float:
        """L2 norm of the flat fp32 master parameters: one native reduction over
        the arena on GPU (csrc/optim.hip sumsq_partial_kernel), the divergence
        watchdog's probe -- a NaN / inf anywhere in the model shows up here."""
        flat = self.arena.p32
        if flat.is_cuda:
            from ..ops._ext import native

            return math.sqrt(float(native().sumsq(flat)))
        return float(flat.double().norm())

    def train_step(self, x, y, keep: bool = True):
        """One fwd+bwd+update. Returns (loss, hits) as device tensors (no sync).
        ``keep=False``: with hipGraph replay the returned tensors are the graph's
        own outputs, valid until the next step (no per-step copy kernels)."""
        if getattr(self, "use_graph", False):
            return self._graph_step(x, y, keep)
        with self.timer.time("compute_launch"):
            self.opt.zero_grad()
            logits = self.model(x)
            loss, hits = softmax_cross_entropy(logits, y, self.cfg.label_smoothing)
            loss.backward(unit_grad(loss))
        if self.ddp is not None:
            with self.timer.time("allreduce_wait"):
                self.ddp.synchronize()
        if isinstance(self.opt, Asynchronous):
            self.opt.local_step()
            self.opt.comm_step()
        else:
            with self.timer.time("update"):
                self.opt.step()
        self.step_idx += 1
        return loss.detach(), hits

    @torch.no_grad()
    def evaluate(self, loader, max_batches: int | None = None, per_class: bool = False):
        """Mean loss and accuracy over ALL test batches (reference used the last batch
        only, main.py:127); restores train mode afterwards (D6).

        ``per_class``: also return the [C, C] confusion matrix (rows = true class),
        from which :func:`~..utils.metrics.classification_report` prints the
        reference's verbose per-class precision/recall/F1 table (main.py:127-131).
        """
        was = self.model.training
        self.model.eval()
        tot_loss = torch.zeros((), device=self.device)
        tot_hits = torch.zeros((), device=self.device, dtype=torch.int64)
        c = self.num_classes
        conf = torch.zeros(c * c, device=self.device, dtype=torch.int64) if per_class else None
        n = 0
        nb = 0
        with fold_session():                 # eval BatchNorms folded into their convs once
            for xb, yb in loader:
                xb, yb = self.prepare(xb, yb)
                out = self.model(xb)
                loss, hits = softmax_cross_entropy(out, yb)
                tot_loss += loss.float() * yb.numel()
                tot_hits += hits.to(torch.int64)
                if conf is not None:
                    pred = out.float().argmax(1)
                    # rows with an ignored / out-of-range label are skipped, as the
                    # loss kernel skips them (bincount rejects negative indices)
                    ok = (yb >= 0) & (yb < c)
                    conf += torch.bincount((yb * c + pred)[ok], minlength=c * c)
                n += yb.numel()
                nb += 1
                if max_batches and nb >= max_batches:
                    break
        self.model.train(was)
        if n == 0:
            res = (float("nan"), float("nan"))
        else:
            res = ((tot_loss / n).item(), tot_hits.item() / n)
        if per_class:
            return (*res, conf.view(c, c).cpu())
        return res

    def set_lr(self, lr: float):
        for g in self.opt.param_groups:
            g["lr"] = lr

    def finish(self):
        if isinstance(self.opt, Asynchronous):
            self.opt.finish()


def _payload(cfg: TrainConfig, info: DistInfo) -> str:
    if cfg.payload != "auto":
        return cfg.payload
    return "rccl" if info.backend == "nccl" else "gloo"


def run_server(cfg: TrainConfig, info: DistInfo, ps_groups):
    """Rank 0 in the central topology (reference main.py:135-138)."""
    ctrl, pairs = ps_groups
    model, _, _ = build_model(cfg.model, cfg.num_classes)
    payload = _payload(cfg, info)
    server = ParameterServer(model=model, control_group=ctrl, pair_groups=pairs,
                             payload=payload,
                             device=info.device if payload == "rccl" else "cpu",
                             checkpoint_path=cfg.checkpoint,
                             checkpoint_every=cfg.checkpoint_every,
                             worker_timeout=cfg.ps_worker_timeout or None,
                             delta_scale=cfg.delta_scale)
    ps_path = _ps_resume_path(cfg)
    if ps_path:
        server.load_checkpoint(ps_path)
    elif cfg.ps_resume:
        raise FileNotFoundError(f"--ps-resume {cfg.ps_resume}: no parameter-server checkpoint")
    stats = server.run()
    if cfg.verbose:
        print(f"[ps] finished: {stats}", flush=True)
    return stats


def run_training(cfg: TrainConfig, info: DistInfo):
    """Entry point for every rank. Returns a result dict (worker) or PS stats."""
    ps_groups = None
    central = cfg.mode == "asgd" and cfg.ps == "central" and info.is_distributed
    if central:
        ps_groups = make_ps_groups(0, _payload(cfg, info))
    # start-up checks every rank joins: ranks reached by a collective, distinct
    # devices on RCCL, every (PS, worker) payload communicator answering
    pf = preflight(info, None, ps_groups[1] if ps_groups else None, 0)
    if cfg.verbose and info.rank == 0 and info.is_distributed:
        print(f"[preflight] {pf}", flush=True)
    if central and info.rank == 0:
        return {"role": "ps", "preflight": pf, **run_server(cfg, info, ps_groups)}
    w = Worker(cfg, info, ps_groups)
    tr, te, source = get_datasets(cfg.dataset, cfg.data_dir, w.input_shape, w.num_classes,
                                  cfg.n_train, cfg.n_test, seed=cfg.seed)
    # every worker sees the full dataset in its own shuffle order (reference has no
    # DistributedSampler, main.py:27); sync-DP shards by rank instead.
    if cfg.mode == "sync" and info.is_distributed:
        idx = list(range(info.rank, len(tr), info.world_size))
        tr = torch.utils.data.Subset(tr, idx)
    train_loader, test_loader = make_loaders(tr, te, cfg.batch_size, cfg.test_batch_size,
                                             shuffle_seed=cfg.seed + info.rank)
    log = IterationLog()
    log_phases = bool(cfg.log_interval)
    meter = Throughput(sync_cuda=w.device.type == "cuda")
    base_lr = cfg.lr
    done = False
    t_start = time.perf_counter()
    for epoch in range(cfg.epochs):
        if cfg.lr_schedule == "inv_epoch":
            w.set_lr(base_lr / (epoch + 1))
        if cfg.verbose and info.rank <= 1:
            print(f"Training for epoch {epoch}", flush=True)
        for i, (xb, yb) in enumerate(train_loader):
            xb, yb = w.prepare(xb, yb)
            loss, hits = w.train_step(xb, yb)
            meter.add(yb.numel())
            row = log.append(epoch, i, loss)
            if cfg.log_interval and i % cfg.log_interval == 0 and i > 0:
                row["samples_per_sec"] = meter.rate()
                row["param_norm"] = w.param_norm()
                if cfg.divergence_check and not math.isfinite(row["param_norm"]):
                    raise DivergenceError(
                        f"rank {info.rank}: non-finite parameters at epoch {epoch} iteration {i} "
                        f"(loss {float(loss):.4g}); lower --lr or pass --no-divergence-check")
                if cfg.evaluate:
                    row["test_loss"], row["test_accuracy"] = w.evaluate(test_loader)
                log.flush_pending()
                if cfg.verbose:
                    print("Timestamp: {timestamp} | Iteration: {iteration:6} | "
                          "Loss: {training_loss:6.4f} | Test Loss: {tl} | Test Accuracy: {ta} | "
                          "samples/s: {sps:.1f}".format(
                              tl=_fmt(row.get("test_loss")), ta=_fmt(row.get("test_accuracy")),
                              sps=row["samples_per_sec"], **row), flush=True)
            if cfg.checkpoint and cfg.checkpoint_every and w.step_idx % cfg.checkpoint_every == 0:
                ckpt.save_worker_checkpoint(_worker_ckpt(cfg, info), w.model, w.opt, w.step_idx)
            if log_phases and i % cfg.log_interval == 0 and i > 0:
                row.update({f"{k}_ms": v["mean_ms"] for k, v in w.timer.summary().items()})
            if cfg.max_steps and w.step_idx >= cfg.max_steps:
                done = True
                break
        if cfg.evaluate and not done:
            vl, va, conf = w.evaluate(test_loader, per_class=True)
            if cfg.verbose:
                print(f"epoch {epoch}: lr {w.opt.param_groups[0]['lr']:.5g} "
                      f"test loss {vl:.4f} test accuracy {va:.4f}", flush=True)
                # the reference's verbose eval prints sklearn's per-class report
                # (/root/reference/example/main.py:127-131)
                print(classification_report(conf), flush=True)
        if done:
            break
    w.finish()
    elapsed = time.perf_counter() - t_start
    final = w.evaluate(test_loader) if cfg.evaluate else (float("nan"), float("nan"))
    if cfg.checkpoint:
        ckpt.save_worker_checkpoint(_worker_ckpt(cfg, info), w.model, w.opt, w.step_idx)
    from ..utils.metrics import log_path

    path = log_path(cfg.mode == "single" and not info.is_distributed,
                    w.device.type == "cuda", info.rank, cfg.log_dir)
    log.to_csv(path)
    res = {"role": "worker", "rank": info.rank, "steps": w.step_idx, "elapsed_s": elapsed,
           "samples_per_sec": meter.rate(), "test_loss": final[0], "test_accuracy": final[1],
           "data": source, "log": path, "preflight": pf}
    if isinstance(w.opt, Asynchronous):
        res.update(w.opt.stats())
    res["phases"] = w.timer.summary()
    if cfg.verbose:
        print(f"[worker {info.rank}] {res}", flush=True)
    return res


def _worker_ckpt(cfg, info):
    return ckpt.worker_checkpoint_path(cfg.checkpoint, info.rank)


def _agree_on_resume(have: bool, info: DistInfo):
    """Collective check that every rank found (or did not find) its worker
    checkpoint; raises on disagreement instead of hanging in the restore."""
    dev = info.device if info.backend == "nccl" else torch.device("cpu")
    t = torch.tensor([1.0 if have else 0.0, 0.0 if have else 1.0], device=dev)
    dist.all_reduce(t)
    n_have, n_miss = int(round(float(t[0]))), int(round(float(t[1])))
    if n_have and n_miss:
        raise RuntimeError(
            f"resume: {n_have} rank(s) found their worker checkpoint and {n_miss} did not "
            f"(this is rank {info.rank}, {'found' if have else 'missing'}): the sharded / "
            "sync topologies restore collectively; supply every <base>.worker<r>.pt or none")


def _worker_resume_path(base: str, rank: int) -> str | None:
    """``<base>.worker<rank>.pt`` if present, else ``base`` when it is itself a worker
    checkpoint, else ``None`` (e.g. only a PS checkpoint: the worker starts fresh
    and adopts the PS parameters at its first pull)."""
    cand = ckpt.worker_checkpoint_path(base, rank)
    if os.path.exists(cand):
        return cand
    if os.path.exists(base) and ckpt.checkpoint_kind(base) == "worker":
        return base
    return None


def _ps_resume_path(cfg) -> str | None:
    for p in (cfg.ps_resume, cfg.resume):
        if p and os.path.exists(p) and ckpt.checkpoint_kind(p) == "ps":
            return p
    return None


def _fmt(v):
    return "   n/a" if v is None or (isinstance(v, float) and math.isnan(v)) else f"{v:6.4f}"


def config_dict(cfg: TrainConfig) -> dict:
    return asdict(cfg)
