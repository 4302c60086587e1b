"""End-to-end training on one MI355X through the native kernels."""
import math
import pytest

import torch

pytestmark = pytest.mark.gpu


def _worker(model, mode="asgd", ps="local", batch=32, lr=0.05, **kw):
    from distributed_ml_pytorch_amd.runtime.dist import DistInfo
    from distributed_ml_pytorch_amd.runtime.trainer import TrainConfig, Worker

    cfg = TrainConfig(model=model, batch_size=batch, mode=mode, ps=ps, lr=lr, evaluate=False,
                      verbose=False, **kw)
    return Worker(cfg, DistInfo(device=torch.device("cuda", 0)))


@pytest.mark.parametrize("model", ["resnet18", "alexnet", "lenet", "vit_tiny", "mlp"])
def test_loss_decreases_on_fixed_batch(model):
    w = _worker(model, n_push=5, n_pull=5)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(32, *w.input_shape, generator=g)
    y = torch.randint(0, w.num_classes, (32,), generator=g)
    x, y = w.prepare(x, y)
    losses = []
    for _ in range(30):
        loss, _ = w.train_step(x, y)
        losses.append(float(loss.float()))
    w.finish()
    assert all(l == l for l in losses)
    assert min(losses[-5:]) < losses[0], losses


def test_native_path_is_used_for_resnet():
    """The bf16 GPU path must go through the HIP kernels (no silent fallback)."""
    from distributed_ml_pytorch_amd.ops import _ext

    assert _ext.available()
    w = _worker("resnet18")
    x, y = w.prepare(torch.randn(8, 3, 32, 32), torch.randint(0, 10, (8,)))
    loss, _ = w.train_step(x, y)
    assert "_native" in (_ext.so_path() or "")
    assert w.arena.w16 is not None and w.arena.w16.dtype == torch.bfloat16


def test_asgd_matches_fp32_oracle_math():
    """One ASGD step on GPU == reference math p -= lr*g, acc -= lr*g (Asynchronous.py:54-68)."""
    w = _worker("mlp", n_push=100, n_pull=100, lr=0.1)
    x, y = w.prepare(torch.randn(16, 1, 28, 28), torch.randint(0, 10, (16,)))
    p0 = w.arena.p32.clone()
    acc0 = w.opt.acc.clone()
    w.opt.zero_grad()
    out = w.model(x)
    from distributed_ml_pytorch_amd.ops.functional import softmax_cross_entropy

    loss, _ = softmax_cross_entropy(out, y)
    loss.backward()
    g = w.arena.g32.clone()
    w.opt.n_push = 10 ** 9   # no push this step (idx 0 would push)
    w.opt.idx = 1
    w.opt.step()
    torch.testing.assert_close(w.arena.p32, p0 - 0.1 * g)
    torch.testing.assert_close(w.opt.acc, acc0 - 0.1 * g)
    torch.testing.assert_close(w.arena.w16, w.arena.p32.to(torch.bfloat16), rtol=0, atol=0)


def test_sync_single_process_and_modes():
    for mode in ("sync", "single"):
        w = _worker("resnet18", mode=mode)
        x, y = w.prepare(torch.randn(16, 3, 32, 32), torch.randint(0, 10, (16,)))
        l0, _ = w.train_step(x, y)
        for _ in range(5):
            l1, _ = w.train_step(x, y)
        assert float(l1) < float(l0)


def test_bench_script_runs():
    import json
    import subprocess
    import sys
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "3",
                        "--warmup", "1", "--batch", "32"], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["unit"] == "samples/s"


def test_graph_replay_matches_eager():
    """hipGraph-captured steps train the same model as eager steps (same data, same init)."""
    import copy

    torch.manual_seed(0)
    g = torch.Generator().manual_seed(1)
    xs = [torch.randn(16, 3, 32, 32, generator=g) for _ in range(6)]
    ys = [torch.randint(0, 10, (16,), generator=g) for _ in range(6)]
    res = {}
    for graph in (False, True):
        torch.manual_seed(0)
        w = _worker("resnet18", n_push=3, n_pull=3, lr=0.01)
        w.enable_graph(graph)
        losses = []
        for x, y in zip(xs, ys):
            x, y = w.prepare(x, y)
            loss, _ = w.train_step(x, y)
            losses.append(float(loss.float()))
        w.finish()
        res[graph] = (losses, w.arena.p32.clone(), w.step_idx)
    le, pe, ne = res[False]
    lg, pg, ng = res[True]
    assert ne == ng == 6
    # wgrad and the BN statistics use fp32 atomics (order-dependent sums), so
    # the two runs differ by rounding that training amplifies: tolerance
    assert max(abs(a - b) for a, b in zip(le, lg)) < 5e-2, (le, lg)
    assert float((pe - pg).norm() / pe.norm()) < 1e-2


def test_back_to_back_graph_replays_stay_finite():
    """Bench-shaped ResNet-18 (bs 512) hipGraph replays issued back to back with no
    host sync in between train like eager steps.  Regression: the grad-arena zero
    as a captured hipMemsetAsync node was not ordered behind the previous replay
    and the trajectory went non-finite within tens of steps (now a fill kernel)."""
    from distributed_ml_pytorch_amd.utils.data import DeviceBatchPool

    res = {}
    for graph in (True, False):
        torch.manual_seed(0)
        w = _worker("resnet18", n_push=1000, n_pull=1000, lr=0.05, batch=512)
        w.enable_graph(graph)
        pool = DeviceBatchPool(512, w.input_shape, w.num_classes, w.device, n_batches=4,
                               dtype=w.compute_dtype, seed=0)
        losses = []
        for _ in range(40):
            x, y = pool.next()
            loss, _ = w.train_step(x, y)       # no .item(): replays queue back to back
            losses.append(loss)
        torch.cuda.synchronize()
        res[graph] = ([float(v.float()) for v in losses], w.param_norm())
        w.finish()
    lg, ng = res[True]
    le, ne = res[False]
    assert all(math.isfinite(v) and v < 10 for v in lg), lg
    assert math.isfinite(ng) and abs(ng - ne) / ne < 1e-3, (ng, ne)
    assert abs(lg[-1] - le[-1]) < 0.1, (lg[-5:], le[-5:])


def _nccl_world1():
    import os
    import socket

    import torch.distributed as dist

    if dist.is_initialized():
        return
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1)


def test_rccl_sharded_ps_and_bucketed_allreduce_paths():
    """Exercise the real RCCL calls (reduce-scatter/all-gather on a side stream,
    bucketed all-reduce from backward hooks) with a world-size-1 NCCL group."""
    import torch.distributed as dist

    from distributed_ml_pytorch_amd.models import build_model
    from distributed_ml_pytorch_amd.parallel.arena import attach_arena
    from distributed_ml_pytorch_amd.parallel.asgd import Asynchronous
    from distributed_ml_pytorch_amd.parallel.clients import LocalPSClient, ShardedPSClient
    from distributed_ml_pytorch_amd.parallel.ddp import BucketedAllReduce, FusedSGD

    _nccl_world1()
    try:
        g = torch.Generator().manual_seed(3)
        xs = [torch.randn(16, 3, 32, 32, generator=g) for _ in range(5)]
        ys = [torch.randint(0, 10, (16,), generator=g) for _ in range(5)]
        finals = {}
        for kind in ("local", "sharded"):
            torch.manual_seed(0)
            m, _, _ = build_model("resnet18")
            m = m.cuda()
            client = LocalPSClient(staleness=1) if kind == "local" else \
                ShardedPSClient(staleness=1, force_collectives=True)
            opt = Asynchronous(m.parameters(), lr=0.05, n_push=2, n_pull=2, model=m,
                               client=client)
            from distributed_ml_pytorch_amd.ops.functional import softmax_cross_entropy

            for x, y in zip(xs, ys):
                x = x.cuda().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
                opt.zero_grad()
                loss, _ = softmax_cross_entropy(m(x), y.cuda())
                loss.backward()
                opt.step()
            opt.finish()
            torch.cuda.synchronize()
            finals[kind] = opt.arena.p32.clone()
        # same math through RCCL (world 1) as through the in-process PS
        rel = float((finals["local"] - finals["sharded"]).norm() / finals["local"].norm())
        assert rel < 1e-2, rel
        # bucketed all-reduce through RCCL: grads unchanged at world 1
        torch.manual_seed(0)
        m, _, _ = build_model("resnet18")
        m = m.cuda()
        arena = attach_arena(m)
        ddp = BucketedAllReduce(arena, bucket_mb=4, force_collectives=True)
        opt = FusedSGD(list(m.parameters()), arena, lr=0.05)
        x = xs[0].cuda().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        from distributed_ml_pytorch_amd.ops.functional import softmax_cross_entropy

        opt.zero_grad()
        loss, _ = softmax_cross_entropy(m(x), ys[0].cuda())
        loss.backward()
        launched = sum(w is not None for w in ddp.works)
        ddp.synchronize()
        assert ddp.num_buckets >= 3 and launched >= 1   # some buckets fired during backward
        assert torch.isfinite(arena.g32).all()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("model", ["resnet18", "vit_tiny", "alexnet", "resnet50"])
def test_fp32_gpu_mode_is_an_oracle(model):
    """``--dtype fp32`` on the GPU: every op on PyTorch's fp32 kernels (no bf16
    shadow), same model / optimizer / PS.  Its first-step loss and parameters
    after a few ASGD steps track the bf16 native run within bf16 noise."""
    runs = {}
    for dt in ("fp32", "bf16"):
        torch.manual_seed(0)
        w = _worker(model, n_push=2, n_pull=2, lr=0.02, dtype=dt, seed=3)
        assert (w.arena.w16 is None) == (dt == "fp32")
        g = torch.Generator().manual_seed(0)
        x = torch.randn(16, *w.input_shape, generator=g)
        y = torch.randint(0, w.num_classes, (16,), generator=g)
        x, y = w.prepare(x, y)
        losses = [float(w.train_step(x, y)[0].float()) for _ in range(4)]
        w.finish()
        torch.cuda.synchronize()
        runs[dt] = (losses, w.arena.p32.clone())
    (l32, p32), (l16, p16) = runs["fp32"], runs["bf16"]
    assert all(v == v for v in l32)
    assert abs(l32[0] - l16[0]) < 0.05 * abs(l32[0]) + 0.02, (l32, l16)
    rel = float((p16 - p32).norm() / p32.norm())
    # ResNet-50 from a random init is chaotic: stock autocast-bf16's gradients are
    # ~1.3 off fp32 there (profiles/grad_parity_resnet50_r2.txt); 4 steps leave
    # ~3.3 % parameter drift with or without the fused stem (DMP_BN_POOL_FUSE=0/1)
    assert rel < (5e-2 if model == "resnet50" else 1e-2), rel


def test_rccl_world1_device_async_shards_and_bf16_wire():
    """World-size-1 NCCL group: the non-lock-step sharded PS runs its GPU
    transport (device-resident shard, PS-stream apply / snapshot, per-slice
    pull landing) and the collective sharded PS its bf16 wire (all-to-all of
    bf16 slices + fp32 apply); both track the in-process PS run."""
    import torch.distributed as dist

    from distributed_ml_pytorch_amd.models import build_model
    from distributed_ml_pytorch_amd.ops.functional import softmax_cross_entropy
    from distributed_ml_pytorch_amd.parallel.asgd import Asynchronous
    from distributed_ml_pytorch_amd.parallel.async_sharded import AsyncShardedPSClient
    from distributed_ml_pytorch_amd.parallel.clients import LocalPSClient, ShardedPSClient

    _nccl_world1()
    try:
        g = torch.Generator().manual_seed(5)
        xs = [torch.randn(16, 3, 32, 32, generator=g) for _ in range(6)]
        ys = [torch.randint(0, 10, (16,), generator=g) for _ in range(6)]
        finals = {}
        for kind in ("local", "async", "sharded_bf16"):
            torch.manual_seed(0)
            m, _, _ = build_model("resnet18")
            m = m.cuda()
            client = {"local": lambda: LocalPSClient(staleness=1),
                      "async": lambda: AsyncShardedPSClient(staleness=1),
                      "sharded_bf16": lambda: ShardedPSClient(
                          staleness=1, force_collectives=True, wire_dtype=torch.bfloat16)}[kind]()
            opt = Asynchronous(m.parameters(), lr=0.05, n_push=2, n_pull=2, model=m,
                               client=client)
            for x, y in zip(xs, ys):
                x = x.cuda().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
                opt.zero_grad()
                loss, _ = softmax_cross_entropy(m(x), y.cuda())
                loss.backward()
                opt.step()
            opt.finish()
            torch.cuda.synchronize()
            finals[kind] = (opt.arena.p32.clone(), opt.stats())
        ref = finals["local"][0]
        for kind in ("async", "sharded_bf16"):
            rel = float((finals[kind][0] - ref).norm() / ref.norm())
            assert rel < 1e-2, (kind, rel)
        st = finals["async"][1]
        assert st["pushes"] == 3 and st["pulls"] == 3 and st["shard_version"] == 3
        assert st["payload"] == "rccl"
    finally:
        dist.destroy_process_group()


def _det_run(model, steps=6, mode="asgd", graph=False):
    w = _worker(model, mode=mode, batch=16, n_push=2, n_pull=3, deterministic=True)
    if graph:
        w.enable_graph(True)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(16, *w.input_shape, generator=g)
    y = torch.randint(0, w.num_classes, (16,), generator=g)
    x, y = w.prepare(x, y)
    losses = [float(w.train_step(x, y)[0].float()) for _ in range(steps)]
    w.finish()
    torch.cuda.synchronize()
    return losses, w.arena.p32.clone(), w.compute_dtype


@pytest.mark.parametrize("model,mode", [("resnet18", "asgd"), ("vit_tiny", "sync")])
def test_deterministic_mode_is_bitwise_reproducible(model, mode):
    """--deterministic: two runs of the same steps give bitwise-equal losses and
    parameters (runtime/determinism.py; the bf16 native path sums split reductions
    with fp32 atomics and is only reproducible to rounding)."""
    try:
        l1, p1, dt = _det_run(model, mode=mode)
        l2, p2, _ = _det_run(model, mode=mode)
        assert torch.are_deterministic_algorithms_enabled()
    finally:
        torch.use_deterministic_algorithms(False)
        torch.backends.cudnn.deterministic = False
    assert dt == torch.float32
    assert all(l == l for l in l1), l1
    assert l1 == l2, (l1, l2)
    assert torch.equal(p1, p2)


def test_vit_native_gradients_match_fp32():
    """One ViT-tiny backward on the native bf16 path (fused add+LayerNorm, the
    stream-gradient LayerNorm of block 0, fused MLP / attention) against the same
    weights on PyTorch's fp32 kernels: every parameter's gradient within bf16 noise."""
    from distributed_ml_pytorch_amd.ops.functional import softmax_cross_entropy

    grads = {}
    for dt in ("fp32", "bf16"):
        w = _worker("vit_tiny", n_push=100, n_pull=100, dtype=dt, seed=5)
        g = torch.Generator().manual_seed(0)
        x = torch.randn(8, *w.input_shape, generator=g)
        y = torch.randint(0, w.num_classes, (8,), generator=g)
        x, y = w.prepare(x, y)
        w.opt.zero_grad()
        loss, _ = softmax_cross_entropy(w.model(x), y)
        loss.backward()
        torch.cuda.synchronize()
        grads[dt] = {n: p.grad.detach().float().clone() for n, p in w.model.named_parameters()}
    bad = {}
    for n, ref in grads["fp32"].items():
        got = grads["bf16"][n]
        rel = float((got - ref).norm() / (ref.norm() + 1e-12))
        if rel > 5e-2:
            bad[n] = rel
    assert not bad, bad


def test_local_ps_side_stream_matches_compute_stream(monkeypatch):
    """LocalPSClient with the PS apply / pull snapshot on the side stream (event-ordered,
    DMP_LOCAL_PS_SIDE=1) trains bitwise like the compute-stream placement: in the
    deterministic mode both runs must agree exactly (push / pull cadence 2 / 3 steps)."""
    from distributed_ml_pytorch_amd.parallel.clients import LocalPSClient

    runs = {}
    try:
        for side in (False, True):
            monkeypatch.setattr(LocalPSClient, "SIDE", side)
            runs[side] = _det_run("resnet18", steps=7)
    finally:
        torch.use_deterministic_algorithms(False)
        torch.backends.cudnn.deterministic = False
    (l0, p0, _), (l1, p1, _) = runs[False], runs[True]
    assert all(v == v for v in l0), l0
    assert l0 == l1, (l0, l1)
    assert torch.equal(p0, p1)
