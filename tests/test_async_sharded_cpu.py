"""Non-lock-step sharded parameter server (parallel/async_sharded.py), gloo on CPU.

* every delta reaches its shard exactly once: after all ranks finish, the
  concatenated shards equal init + the sum of every rank's pushes;
* no lock-step: a rank that stalls does not stop another rank's pushes and
  pulls (its shard server thread keeps answering), while the collective
  ShardedPSClient blocks the fast rank until the late one joins.
"""
import time

import pytest
import torch
import torch.distributed as dist
import torch.nn as nn

from test_dist_cpu import _run

pytestmark = pytest.mark.slow


def _grad(rank, k, like):
    g = torch.Generator().manual_seed(1000 * rank + k)
    return torch.randn(like.shape, generator=g)


def _sum_of_pushes(world, steps, lr):
    torch.manual_seed(0)
    m = nn.Linear(6, 5)
    from distributed_ml_pytorch_amd.parallel.arena import attach_arena

    arena = attach_arena(m, shadow_dtype=None)
    init = arena.p32.clone()
    # replay every rank's deltas on the same arena layout
    for r in range(world):
        for k in range(steps):
            for p in m.parameters():
                p.grad.copy_(_grad(r, k, p))
            init.add_(arena.g32, alpha=-lr)
    return init


def _math(rank, world, steps, lr):
    from distributed_ml_pytorch_amd.parallel.async_sharded import AsyncShardedPSClient
    from distributed_ml_pytorch_amd.parallel.asgd import Asynchronous

    torch.manual_seed(0)            # identical init (rank 0's is broadcast anyway)
    m = nn.Linear(6, 5)
    opt = Asynchronous(m.parameters(), lr=lr, n_push=1, n_pull=3, model=m,
                       client=AsyncShardedPSClient(staleness=1), shadow_dtype=None)
    for k in range(steps):
        opt.zero_grad()
        for p in m.parameters():
            p.grad.copy_(_grad(rank, k, p))
        opt.step()
    opt.finish()
    st = opt.stats()
    shards = [torch.zeros_like(opt.client.master) for _ in range(world)]
    dist.all_gather(shards, opt.client.master)
    return {"master": torch.cat(shards).numpy(), "stats": st}


def test_async_sharded_every_push_applied_once():
    world, steps, lr = 3, 7, 0.1
    out = _run(_math, world, steps, lr)
    want = _sum_of_pushes(world, steps, lr)
    for r in range(world):
        got = torch.from_numpy(out[r]["master"])
        torch.testing.assert_close(got[: want.numel()], want, rtol=1e-5, atol=1e-5)
        st = out[r]["stats"]
        # this shard applied its own 7 pushes in-process + 7 from each other rank
        assert st["shard_version"] == world * steps
        assert st["shard_applied"] == world * steps
        assert st["shard_counts"]["GradientUpdate"] == (world - 1) * steps
        assert st["shard_counts"]["ParameterRequest"] == (world - 1) * len(range(0, steps, 3))
        assert st["pushes"] == steps


def _math_delayed(rank, world, steps, lr, delay):
    """n_push=1 < n_pull=4 with one slow rank: every ring slot of the link path
    (parallel/links.py) is reused many times while the slow peer's pushes and
    pull requests arrive late and interleaved with the fast ranks'."""
    from distributed_ml_pytorch_amd.parallel.async_sharded import AsyncShardedPSClient
    from distributed_ml_pytorch_amd.parallel.asgd import Asynchronous

    torch.manual_seed(0)
    m = nn.Linear(6, 5)
    opt = Asynchronous(m.parameters(), lr=lr, n_push=1, n_pull=4, model=m,
                       client=AsyncShardedPSClient(staleness=2), shadow_dtype=None)
    for k in range(steps):
        if rank == world - 1:
            time.sleep(delay)
        opt.zero_grad()
        for p in m.parameters():
            p.grad.copy_(_grad(rank, k, p))
        opt.step()
    opt.finish()
    st = opt.stats()
    shards = [torch.zeros_like(opt.client.master) for _ in range(world)]
    dist.all_gather(shards, opt.client.master)
    return {"master": torch.cat(shards).numpy(), "stats": st}


def test_async_sharded_link_rings_with_a_slow_peer():
    world, steps, lr = 3, 12, 0.1
    out = _run(_math_delayed, world, steps, lr, 0.05)
    want = _sum_of_pushes(world, steps, lr)
    n_pulls = len(range(0, steps, 4))
    for r in range(world):
        got = torch.from_numpy(out[r]["master"])
        # every delta applied exactly once, none lost to a reused slot
        torch.testing.assert_close(got[: want.numel()], want, rtol=1e-5, atol=1e-5)
        st = out[r]["stats"]
        assert st["shard_version"] == world * steps
        assert st["shard_applied"] == world * steps
        links = st["shard_links"]
        assert links["recv"] == (world - 1) * steps
        assert links["reused"] >= (world - 1) * (steps - 2)     # depth-2 rings
        assert links["sends"] == (world - 1) * n_pulls
        # landed versions: one per shard, the base version is their minimum
        assert len(st["shard_versions"]) == world
        assert st["version"] == min(st["shard_versions"])
        assert st["shard_staleness_max"] >= 0


def _straggler(rank, world, kind, pause):
    from distributed_ml_pytorch_amd.parallel.async_sharded import AsyncShardedPSClient
    from distributed_ml_pytorch_amd.parallel.asgd import Asynchronous
    from distributed_ml_pytorch_amd.parallel.clients import ShardedPSClient

    torch.manual_seed(0)
    m = nn.Linear(32, 16)
    client = AsyncShardedPSClient(staleness=1) if kind == "async" else ShardedPSClient(staleness=1)
    opt = Asynchronous(m.parameters(), lr=0.01, n_push=1, n_pull=1, model=m, client=client,
                       shadow_dtype=None)
    dist.barrier()
    if rank == 1:
        time.sleep(pause)           # the straggler: its worker is stuck for `pause` s
    t0 = time.monotonic()
    for k in range(20):
        opt.zero_grad()
        for p in m.parameters():
            p.grad.copy_(_grad(rank, k, p))
        opt.step()
    elapsed = time.monotonic() - t0
    opt.finish()
    return {"elapsed": elapsed}


def test_async_sharded_is_not_lock_step():
    pause = 3.0
    out = _run(_straggler, 2, "async", pause)
    # rank 0 pushed and pulled 20 times while rank 1 was paused
    assert out[0]["elapsed"] < pause / 2, out


def test_collective_sharded_is_lock_step():
    """Contrast: the collective sharded PS makes the fast rank wait for the late one."""
    pause = 3.0
    out = _run(_straggler, 2, "collective", pause)
    assert out[0]["elapsed"] > pause * 0.8, out
