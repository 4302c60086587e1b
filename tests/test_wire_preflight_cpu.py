"""bf16 wire payloads (Local / Sharded / Central PS clients) against fp32 oracles,
and the multi-rank start-up preflight (device assignment, distinct devices,
observed collective world, pair-communicator ping), on CPU over gloo.

The reference ships raw fp32 deltas and parameters
(/root/reference/asgd/optim/Asynchronous.py:34,49,59); SURVEY §5.8 allows bf16
or fp32 bulk payloads with an fp32 master.  bf16 changes only the bytes on the
wire: the sharded PS must still SUM in fp32 (an all-to-all of bf16 slices added
to the fp32 master one by one, never a bf16 reduce-scatter).
"""
import os
import sys

import pytest
import torch
import torch.distributed as dist
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_dist_cpu import _run  # noqa: E402

from distributed_ml_pytorch_amd.models import build_model  # noqa: E402
from distributed_ml_pytorch_amd.parallel.asgd import Asynchronous  # noqa: E402
from distributed_ml_pytorch_amd.parallel.clients import LocalPSClient  # noqa: E402
from distributed_ml_pytorch_amd.runtime import dist as D  # noqa: E402


def _bf(t):
    return t.to(torch.bfloat16).to(torch.float32)


# ------------------------------------------------------------------ local PS
def test_local_ps_bf16_wire_matches_rounded_oracle():
    """Push = bf16(acc) added to the fp32 master; pull = bf16(master) landed."""
    torch.manual_seed(3)
    m, _, _ = build_model("mlp")
    opt = Asynchronous(m.parameters(), lr=0.05, n_push=2, n_pull=3, model=m,
                       client=LocalPSClient(staleness=0, wire_dtype=torch.bfloat16))
    master = opt.client.master.clone()
    p = opt.arena.p32.clone()
    acc = torch.zeros_like(p)
    for idx in range(7):
        x, y = torch.randn(8, 1, 28, 28), torch.randint(0, 10, (8,))
        opt.zero_grad()
        nn.functional.cross_entropy(m(x), y).backward()
        g = opt.arena.g32.clone()
        opt.step()
        acc -= 0.05 * g
        p -= 0.05 * g
        if idx % 2 == 0:
            master += _bf(acc)
            acc.zero_()
        if idx % 3 == 0:
            p = _bf(master).clone()
    # fp32 rounding differences of the oracle's accumulator can move a handful of
    # bf16 roundings by one bf16 ulp (~4e-3 relative); everything else is exact
    for got, want in ((opt.client.master, master), (opt.arena.p32, p)):
        diff = (got - want).abs()
        assert float(diff.max()) < 1e-5
        assert int((diff > 1e-6).sum()) < 1e-4 * diff.numel()
    assert opt.client.bytes_sent == 4 * opt.arena.numel * 2     # 4 pushes of bf16


# ---------------------------------------------------------------- sharded PS
def _sharded_bf16(rank, world):
    from distributed_ml_pytorch_amd.parallel.clients import ShardedPSClient

    torch.manual_seed(100 + rank)
    m, _, _ = build_model("mlp")
    opt = Asynchronous(m.parameters(), lr=0.1, n_push=2, n_pull=2, model=m,
                       client=ShardedPSClient(staleness=0, wire_dtype=torch.bfloat16))
    p0 = opt.arena.p32.clone()
    torch.manual_seed(rank)
    deltas = []
    for _ in range(4):
        x, y = torch.randn(8, 1, 28, 28), torch.randint(0, 10, (8,))
        opt.zero_grad()
        nn.functional.cross_entropy(m(x), y).backward()
        deltas.append(-0.1 * opt.arena.g32.clone())
        opt.step()
    opt.finish()
    # idx 0 push+pull, idx 2 push+pull (staleness 0): the master holds
    # p0 + sum_r bf16(acc_r) for both pushes, added slice by slice in fp32 in
    # rank order; the pull lands bf16(master)
    pushes = [deltas[0], deltas[1] + deltas[2]]
    n = p0.numel()
    sn = n // world
    lo, hi = rank * sn, (rank + 1) * sn
    mine = [_bf(d) for d in pushes]
    allp = [[torch.zeros_like(d) for _ in range(world)] for d in mine]
    for k, d in enumerate(mine):
        dist.all_gather(allp[k], d)
    master = p0.clone()
    for k in range(2):
        for r in range(world):
            master[lo:hi] += allp[k][r][lo:hi]
    err_master = float((opt.client.master - master[lo:hi]).abs().max())
    shards = [torch.zeros(sn) for _ in range(world)]
    dist.all_gather(shards, master[lo:hi].contiguous())
    want = _bf(torch.cat(shards)) + deltas[3]
    err_p = float((opt.arena.p32 - want).abs().max())
    return err_master, err_p


def test_sharded_ps_bf16_wire_reduces_in_fp32():
    out = _run(_sharded_bf16, 2)
    for r, (em, ep) in out.items():
        assert em < 1e-6, (r, em)
        assert ep < 1e-5, (r, ep)


# ---------------------------------------------------------------- central PS
def _central(rank, world, wire):
    import tempfile

    from distributed_ml_pytorch_amd.runtime.dist import DistInfo
    from distributed_ml_pytorch_amd.runtime.trainer import TrainConfig, run_training

    cfg = TrainConfig(model="mlp", n_train=256, n_test=128, test_batch_size=128, batch_size=32,
                      epochs=1, lr=0.05, n_push=2, n_pull=3, mode="asgd", ps="central",
                      cuda=False, log_interval=0, evaluate=True, verbose=False, seed=5,
                      wire_dtype=wire, log_dir=tempfile.mkdtemp())
    info = DistInfo(rank, world, rank, "gloo", torch.device("cpu"))
    res = run_training(cfg, info)
    return {k: v for k, v in res.items() if isinstance(v, (int, float, str, dict))}


def test_central_ps_bf16_wire_tracks_fp32_run():
    """1 PS + 1 worker (a deterministic schedule): the bf16-wire run's test loss
    stays within bf16 noise of the fp32-wire run; the PS saw the same traffic."""
    f32 = _run(_central, 2, "fp32")
    b16 = _run(_central, 2, "bf16")
    assert f32[0]["counts"] == b16[0]["counts"]
    assert b16[0]["bytes_in"] < f32[0]["bytes_in"]          # bf16 pushes
    assert abs(f32[1]["test_loss"] - b16[1]["test_loss"]) < 0.05, (f32[1], b16[1])
    assert b16[1]["preflight"]["ranks_observed"] == 2


# ---------------------------------------------------------------- preflight
def test_assign_device_rules():
    assert D.assign_device(3, 8, "nccl", 8) == 3
    with pytest.raises(D.PreflightError, match="only 1 visible"):
        D.assign_device(0, 1, "nccl", 2)
    with pytest.raises(D.PreflightError, match="no GPU of its own"):
        D.assign_device(2, 2, "nccl")
    assert D.assign_device(5, 2, "gloo", 8) == 1          # explicit rehearsal sharing
    with pytest.raises(D.PreflightError):
        D.assign_device(0, 0, "nccl")


def test_check_distinct_devices():
    D.check_distinct_devices(["h/a", "h/b", "g/a"])
    with pytest.raises(D.PreflightError, match="ranks 0 and 2"):
        D.check_distinct_devices(["h/a", "h/b", "h/a"])


def _preflight(rank, world):
    info = D.DistInfo(rank, world, rank, "gloo", torch.device("cpu"))
    pairs = {w: dist.new_group([0, w], backend="gloo") for w in range(1, world)}
    return D.preflight(info, None, pairs, 0)


def test_preflight_pings_every_pair():
    out = _run(_preflight, 3)
    assert out[0]["ranks_observed"] == 3 and out[0]["pairs_pinged"] == 2
    assert out[1]["pairs_pinged"] == 1 and out[2]["pairs_pinged"] == 1
    assert out[0]["rccl_ranks"] == 0                     # gloo: no RCCL rank observed
    assert len(out[0]["devices"]) == 3
