"""CPU tests of the framework core: arena, serialization, ASGD math, models, checkpoint, CLI."""
import math
import os

import pytest
import torch
import torch.nn as nn

from distributed_ml_pytorch_amd.models import build_model
from distributed_ml_pytorch_amd.parallel.arena import FlatArena, attach_arena
from distributed_ml_pytorch_amd.parallel.asgd import Asynchronous, DownpourSGD
from distributed_ml_pytorch_amd.parallel.clients import LocalPSClient
from distributed_ml_pytorch_amd.utils.serialization import (ravel_model_params,
                                                            unravel_model_params)


@pytest.mark.parametrize("name,count", [("lenet", 62006), ("alexnet", 2472266),
                                        ("resnet18", 11173962), ("resnet50", 25557032),
                                        ("vit_b16", 86567656)])
def test_param_counts(name, count):
    m, _, _ = build_model(name)
    assert sum(p.numel() for p in m.parameters()) == count


def test_ravel_roundtrip_plain_and_arena():
    m, _, _ = build_model("lenet")
    ref = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    assert torch.equal(ravel_model_params(m), ref)
    unravel_model_params(m, ref * 2)
    assert torch.allclose(ravel_model_params(m), ref * 2)
    arena = attach_arena(m, shadow_dtype=None)
    assert torch.equal(ravel_model_params(m), ref * 2)          # order preserved
    flat = ravel_model_params(m, zero_copy=True)
    assert flat.data_ptr() == arena.p32.data_ptr()              # zero copy
    assert flat.numel() % (64 * 840) == 0
    unravel_model_params(m, ref)
    assert torch.equal(ravel_model_params(m), ref)
    for p in m.parameters():                                    # views into the arena
        assert p.data.untyped_storage().data_ptr() == arena.p32.untyped_storage().data_ptr()
        assert p.grad.untyped_storage().data_ptr() == arena.g32.untyped_storage().data_ptr()


def test_arena_alignment_and_channels_last():
    m, _, _ = build_model("resnet18")
    arena = attach_arena(m, shadow_dtype=torch.bfloat16)
    for s in arena.slots:
        assert s.offset % 64 == 0
    conv_w = m.conv1.weight
    assert conv_w.is_contiguous(memory_format=torch.channels_last)
    assert conv_w._dmp_w16.dtype == torch.bfloat16
    assert torch.equal(conv_w._dmp_w16.float(), conv_w.data.to(torch.bfloat16).float())


def _manual_oracle(model, lr, steps, n_push, batches):
    """Pure-PyTorch re-statement of Asynchronous.py:42-71 with an in-process PS."""
    params = list(model.parameters())
    acc = torch.zeros(sum(p.numel() for p in params))
    ps = torch.cat([p.detach().reshape(-1) for p in params]).clone()
    for idx, (x, y) in enumerate(batches[:steps]):
        for p in params:
            p.grad = None
        loss = nn.functional.cross_entropy(model(x), y)
        loss.backward()
        g = torch.cat([p.grad.reshape(-1) for p in params])
        acc.add_(g, alpha=-lr)
        if idx % n_push == 0:
            ps += acc
            acc.zero_()
        with torch.no_grad():
            for p in params:
                p.add_(p.grad, alpha=-lr)
    return torch.cat([p.detach().reshape(-1) for p in params]), ps


def test_asgd_step_matches_oracle_without_pulls():
    torch.manual_seed(0)
    m1, _, _ = build_model("mlp")
    m2, _, _ = build_model("mlp")
    m2.load_state_dict(m1.state_dict())
    batches = [(torch.randn(8, 1, 28, 28), torch.randint(0, 10, (8,))) for _ in range(7)]
    ref_p, ref_ps = _manual_oracle(m1, 0.05, 7, 3, batches)
    client = LocalPSClient(staleness=0)
    opt = Asynchronous(m2.parameters(), lr=0.05, n_push=3, n_pull=10 ** 6, model=m2,
                       client=client)
    for x, y in batches:
        opt.zero_grad()
        nn.functional.cross_entropy(m2(x), y).backward()
        opt.step()   # idx 0 pulls a snapshot equal to the local params (no-op overwrite)
    torch.testing.assert_close(opt.arena.ravel(), ref_p, rtol=1e-5, atol=1e-6)
    ps = opt.client.master
    used = torch.cat([ps[s.offset:s.offset + s.numel] for s in opt.arena.slots])
    torch.testing.assert_close(used, ref_ps, rtol=1e-5, atol=1e-6)
    assert DownpourSGD is Asynchronous


def test_pull_overwrites_local_params_at_step_boundary():
    m, _, _ = build_model("mlp")
    client = LocalPSClient(staleness=0)
    opt = Asynchronous(m.parameters(), lr=0.1, n_push=1000, n_pull=1, model=m, client=client)
    client.master.fill_(0.25)
    x, y = torch.randn(4, 1, 28, 28), torch.randint(0, 10, (4,))
    opt.idx = 1
    opt.zero_grad()
    nn.functional.cross_entropy(m(x), y).backward()
    opt.step()                      # idx 1: pull requested and landed (staleness 0)
    assert torch.all(opt.arena.p32 == 0.25)


def test_staleness_bound_delays_landing():
    m, _, _ = build_model("mlp")
    client = LocalPSClient(staleness=2)
    opt = Asynchronous(m.parameters(), lr=0.0, n_push=1000, n_pull=1000, model=m,
                       client=client)
    client.master.fill_(0.5)
    client.request_pull(step=5)
    client.land_due(6)
    assert not torch.all(opt.arena.p32 == 0.5)
    client.land_due(7)
    assert torch.all(opt.arena.p32 == 0.5)


def test_debug_landing_rejects_a_pull_inside_a_step(monkeypatch):
    """with DMP_DEBUG_LANDING=1 a pulled snapshot landing between
    zero_grad and local_step (mid forward/backward) is an error; the normal
    step-boundary landing of Asynchronous.step passes."""
    monkeypatch.setenv("DMP_DEBUG_LANDING", "1")
    m, _, _ = build_model("mlp")
    client = LocalPSClient(staleness=0)
    opt = Asynchronous(m.parameters(), lr=0.1, n_push=1000, n_pull=1, model=m, client=client)
    assert client.debug_landing
    x, y = torch.randn(4, 1, 28, 28), torch.randint(0, 10, (4,))
    opt.zero_grad()
    client.request_pull(step=0)
    with pytest.raises(RuntimeError, match="inside a training step"):
        client.land_due(1)
    nn.functional.cross_entropy(m(x), y).backward()
    opt.step()                      # local_step closes the compute half, then lands
    assert not client.pending


def test_asgd_rejects_bad_args():
    m, _, _ = build_model("mlp")
    with pytest.raises(ValueError):
        Asynchronous(m.parameters(), lr=-1, n_push=1, n_pull=1, model=m)
    with pytest.raises(TypeError):
        Asynchronous(m.parameters(), lr=0.1)


def test_checkpoint_roundtrip(tmp_path):
    from distributed_ml_pytorch_amd.utils import checkpoint as ck

    m, _, _ = build_model("lenet")
    opt = Asynchronous(m.parameters(), lr=0.1, n_push=2, n_pull=2, model=m,
                       client=LocalPSClient())
    opt.acc.normal_()
    opt.idx = 17
    path = str(tmp_path / "w.pt")
    ck.save_worker_checkpoint(path, m, opt, 17)
    m2, _, _ = build_model("lenet")
    opt2 = Asynchronous(m2.parameters(), lr=0.5, n_push=2, n_pull=2, model=m2,
                        client=LocalPSClient())
    step = ck.load_worker_checkpoint(path, m2, opt2)
    assert step == 17 and opt2.idx == 17
    assert torch.equal(opt2.acc, opt.acc)
    assert torch.equal(ravel_model_params(m2), ravel_model_params(m))
    assert opt2.param_groups[0]["lr"] == 0.1
    ck.save_ps_checkpoint(str(tmp_path / "ps.pt"), torch.arange(8.0), 5, {"counts": {"a": 1}})
    flat, ver, counts = ck.load_ps_checkpoint(str(tmp_path / "ps.pt"))
    assert ver == 5 and torch.equal(flat, torch.arange(8.0)) and counts == {"a": 1}


def test_metrics_csv_schema(tmp_path):
    from distributed_ml_pytorch_amd.utils.metrics import IterationLog, log_path

    log = IterationLog()
    log.append(0, 0, torch.tensor(2.5))
    r = log.append(0, 1, 2.0)
    r["test_loss"], r["test_accuracy"] = 1.0, 0.5
    p = log.to_csv(str(tmp_path / "log" / "node1.csv"))
    head = open(p).readline().strip().split(",")
    assert head[:7] == ["index", "timestamp", "epoch", "iteration", "training_loss", "test_loss",
                        "test_accuracy"]
    assert log_path(True, False, None) == os.path.join("log", "single.csv")
    assert log_path(True, True, None) == os.path.join("log", "gpu.csv")
    assert log_path(False, False, 2) == os.path.join("log", "node2.csv")


def test_cli_single_process(tmp_path):
    from distributed_ml_pytorch_amd.cli import main

    res = main(["--no-distributed", "--model", "mlp", "--epochs", "1", "--n-train", "512",
                "--n-test", "128", "--test-batch-size", "128", "--log-interval", "4",
                "--lr", "0.05", "--log-dir", str(tmp_path / "log")])
    assert res["steps"] == 8
    assert os.path.exists(tmp_path / "log" / "single.csv")
    assert res["test_accuracy"] > 0.3     # learnable synthetic data


def test_divergence_watchdog_halts_and_can_be_disabled(tmp_path):
    """A blown-up learning rate makes the parameters non-finite: the log-interval
    watchdog (arena norm) halts with DivergenceError; --no-divergence-check keeps
    the reference's keep-going behaviour and logs the norm column."""
    import csv

    from distributed_ml_pytorch_amd.cli import main
    from distributed_ml_pytorch_amd.runtime.trainer import DivergenceError

    def argv(lr, log):
        return ["--no-distributed", "--model", "mlp", "--epochs", "1", "--n-train", "512",
                "--n-test", "128", "--log-interval", "4", "--lr", lr,
                "--log-dir", str(tmp_path / log), "--no-eval"]

    with pytest.raises(DivergenceError):
        main(argv("1e30", "log"))
    res = main(argv("1e30", "log") + ["--no-divergence-check"])
    assert res["steps"] == 8
    rows = list(csv.DictReader(open(tmp_path / "log" / "single.csv")))
    norms = [r["param_norm"] for r in rows if r.get("param_norm")]
    assert norms and not math.isfinite(float(norms[-1]))
    main(argv("0.05", "ok"))
    rows = list(csv.DictReader(open(tmp_path / "ok" / "single.csv")))
    assert all(math.isfinite(float(r["param_norm"])) for r in rows if r.get("param_norm"))


def test_synthetic_data_is_learnable():
    from distributed_ml_pytorch_amd.utils.data import SyntheticImages

    ds = SyntheticImages(256, (1, 28, 28), 10, seed=0)
    ds2 = SyntheticImages(256, (1, 28, 28), 10, seed=1)
    # nearest-template classifier is far above chance
    t = torch.stack([ds.x[ds.y == c].mean(0) for c in range(10)])
    pred = (ds2.x.flatten(1) @ t.flatten(1).t()).argmax(1)
    assert (pred == ds2.y).float().mean() > 0.5


def test_ttl_heldout_split_is_disjoint():
    """bench.py's held-out split: same class templates as the TTL training data,
    no sample in common with it, and a template classifier fitted on the
    training split scores it far above chance (same task)."""
    from distributed_ml_pytorch_amd.utils.data import ttl_pools

    tr, he = ttl_pools(64, (3, 8, 8), 10, "cpu", n_train=6, n_heldout=3,
                       dtype=torch.float32, signal=0.5)
    xtr, ytr = torch.cat(tr.x).flatten(1), torch.cat(tr.y)
    xhe, yhe = torch.cat(he.x).flatten(1), torch.cat(he.y)
    assert xhe.shape == (3 * 64, 3 * 8 * 8)
    # disjoint: no held-out row equals any training row
    d = torch.cdist(xhe, xtr)
    assert float(d.min()) > 1.0
    # same templates: nearest class mean of the TRAINING split classifies held-out
    t = torch.stack([xtr[ytr == c].mean(0) for c in range(10)])
    acc = ((xhe @ t.t()).argmax(1) == yhe).float().mean()
    assert acc > 0.5, acc
    # both pools cover every class
    assert set(yhe.tolist()) == set(range(10)) == set(ytr.tolist())


def test_cifar_binary_reader(tmp_path):
    import numpy as np

    from distributed_ml_pytorch_amd.utils.data import get_datasets

    rng = np.random.default_rng(0)
    for name in [f"data_batch_{i}.bin" for i in range(1, 6)] + ["test_batch.bin"]:
        rec = np.zeros((4, 3073), dtype=np.uint8)
        rec[:, 0] = rng.integers(0, 10, 4)
        rec[:, 1:] = rng.integers(0, 256, (4, 3072))
        rec.tofile(tmp_path / name)
    tr, te, src = get_datasets("cifar10", str(tmp_path))
    assert src == "cifar10" and len(tr) == 20 and len(te) == 4
    x, y = tr[0]
    assert x.shape == (3, 32, 32) and -1.0 <= float(x.min()) and float(x.max()) <= 1.0


def test_fused_sgd_dampening_matches_torch_sgd():
    """Momentum with dampening: the first update seeds the buffer with the raw
    gradient, as torch.optim.SGD does (the zero-initialised buffer
    scaled step 1 by (1 - dampening))."""
    import torch.nn as nn

    from distributed_ml_pytorch_amd.parallel.arena import attach_arena
    from distributed_ml_pytorch_amd.parallel.ddp import FusedSGD

    torch.manual_seed(0)
    m = nn.Sequential(nn.Linear(6, 5), nn.Tanh(), nn.Linear(5, 3))
    ref = nn.Sequential(nn.Linear(6, 5), nn.Tanh(), nn.Linear(5, 3))
    ref.load_state_dict(m.state_dict())
    arena = attach_arena(m, shadow_dtype=None)
    opt = FusedSGD(list(m.parameters()), arena, lr=0.1, momentum=0.9, dampening=0.3)
    ropt = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=0.9, dampening=0.3)
    g = torch.Generator().manual_seed(1)
    for _ in range(4):
        x = torch.randn(8, 6, generator=g)
        for mod, o in ((m, opt), (ref, ropt)):
            o.zero_grad()
            mod(x).pow(2).sum().backward()
            o.step()
    for p, q in zip(m.parameters(), ref.parameters()):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-5, atol=1e-6)


def test_deterministic_flag_plumbing():
    """--deterministic reaches the worker: PyTorch deterministic kernels on, fp32 compute."""
    from distributed_ml_pytorch_amd.cli import build_parser, config_from_args
    from distributed_ml_pytorch_amd.runtime.dist import DistInfo
    from distributed_ml_pytorch_amd.runtime.trainer import Worker

    a = build_parser().parse_args(["--model", "mlp", "--no-distributed", "--deterministic"])
    cfg = config_from_args(a)
    assert cfg.deterministic
    try:
        w = Worker(cfg, DistInfo())
        assert torch.are_deterministic_algorithms_enabled()
        assert w.cfg.dtype == "fp32" and w.compute_dtype == torch.float32
    finally:
        torch.use_deterministic_algorithms(False)
        torch.backends.cudnn.deterministic = False


def test_stream_layer_norm_cpu_matches_two_consumers():
    """ops.functional.stream_layer_norm on CPU: (x, LayerNorm(x)) whose two outputs'
    gradients both reach x (the GPU path forms the sum inside the LN backward)."""
    import torch.nn.functional as F

    from distributed_ml_pytorch_amd.ops.functional import stream_layer_norm

    torch.manual_seed(0)
    x = torch.randn(3, 5, 16, requires_grad=True)
    w = torch.randn(16, requires_grad=True)
    b = torch.randn(16, requires_grad=True)
    h, y = stream_layer_norm(x, w, b, 1e-6)
    (h * 2.0 + y * 3.0).sum().backward()
    x2 = x.detach().clone().requires_grad_(True)
    ref = x2 * 2.0 + F.layer_norm(x2, (16,), w.detach(), b.detach(), 1e-6) * 3.0
    ref.sum().backward()
    torch.testing.assert_close(x.grad, x2.grad)


def test_deferred_residual_mask_helpers():
    """ops/functional.py deferred residual mask: apply_bitmask unpacks bn.hip's
    [pixels, C/8] byte mask (bit k of byte e = NHWC element 8e + k), a tag is
    bound to the tensor's version, and an in-place change is refused."""
    import pytest

    from distributed_ml_pytorch_amd.ops import functional as Fn

    torch.manual_seed(0)
    t = torch.randn(2, 16, 3, 5).contiguous(memory_format=torch.channels_last)
    keep = torch.rand(2, 3, 5, 16) > 0.5                       # NHWC
    packed = (keep.view(-1, 8).to(torch.uint8) << torch.arange(8, dtype=torch.uint8)).sum(
        1).to(torch.uint8)
    out = Fn.apply_bitmask(t, packed)
    assert out.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(out, torch.where(keep.permute(0, 3, 1, 2), t, torch.zeros(())))
    assert Fn.deferred_mask(t) is None and Fn.resolve_deferred(t) is t
    Fn.defer_tag(t, packed)
    assert Fn.deferred_mask(t) is packed
    assert torch.equal(Fn.resolve_deferred(t), out)
    t.add_(1.0)
    with pytest.raises(RuntimeError):
        Fn.deferred_mask(t)


def test_stock_policy_override_nests_and_reaches_other_threads():
    """ops._policy.stock_allowed holds for every thread while the block runs (a CUDA
    backward executes on the autograd engine's device thread), and nests.  (The
    conftest fixture already runs this test inside an allowing block.)"""
    import threading

    from distributed_ml_pytorch_amd.ops._policy import is_allowed, stock_allowed

    outer = is_allowed()
    for on in (False, True):
        with stock_allowed(on):
            seen = []
            t = threading.Thread(target=lambda: seen.append(is_allowed()))
            t.start()
            t.join()
            assert seen == [on] and is_allowed() == on
            with stock_allowed(not on):
                assert is_allowed() == (not on)
            assert is_allowed() == on
    assert is_allowed() == outer
