"""Virtual workers: K model replicas in one process sharing one parameter server
(SURVEY §4 item 6 - the reference's 1 PS + N workers topology, Makefile:13-20, on
one device).  CPU tests run everywhere; the GPU test drives K HIP streams."""
import pytest
import torch


def _run(device, model, k=3, steps=12, batch=32, graph=False, n_push=1, n_pull=3, lr=0.05):
    from distributed_ml_pytorch_amd.parallel.clients import SharedPS
    from distributed_ml_pytorch_amd.runtime.trainer import TrainConfig
    from distributed_ml_pytorch_amd.runtime.virtual import VirtualWorkers
    from distributed_ml_pytorch_amd.utils.data import DeviceBatchPool

    applied = []
    orig = SharedPS.apply

    def spy(self, delta):
        applied.append(delta.detach().to(torch.float32).clone())
        return orig(self, delta)

    SharedPS.apply = spy
    try:
        cfg = TrainConfig(model=model, batch_size=batch, mode="asgd", lr=lr, n_push=n_push,
                          n_pull=n_pull, cuda=device.type == "cuda", evaluate=False,
                          verbose=False)
        vw = VirtualWorkers(cfg, k, device=device)
        init = vw.master().clone()
        # every replica adopted the PS's initial parameters
        for w in vw.workers:
            assert torch.equal(w.arena.p32, init)
        if graph:
            assert vw.enable_graph(True)
        w0 = vw.workers[0]
        dt = w0.compute_dtype if device.type == "cuda" else torch.float32
        pools = [DeviceBatchPool(batch, w0.input_shape, w0.num_classes, device, n_batches=2,
                                 dtype=dt, seed=i, learnable=True, signal=1.0,
                                 channels_last=device.type == "cuda") for i in range(k)]
        losses = []
        for _ in range(steps):
            losses.append([float(l.float()) for l in vw.step([p.next() for p in pools])])
        vw.finish()
        master = vw.master()
        if device.type == "cuda":
            torch.cuda.synchronize()
    finally:
        SharedPS.apply = orig
    return vw, init, master, applied, losses


def _check(vw, init, master, applied, losses, k, steps, n_push):
    # every push of every worker reached the PS, and nothing else changed it
    assert len(applied) == k * ((steps + n_push - 1) // n_push)
    expect = init.clone()
    for d in applied:
        expect += d
    torch.testing.assert_close(master, expect, rtol=1e-5, atol=1e-5)
    assert sum(s["pushes"] for s in vw.stats()) == len(applied)
    first = sum(losses[0]) / k
    last = sum(losses[-1]) / k
    assert all(x == x for row in losses for x in row)
    assert last < first, losses


def test_virtual_workers_cpu():
    k, steps = 3, 12
    out = _run(torch.device("cpu"), "mlp", k=k, steps=steps)
    _check(*out, k=k, steps=steps, n_push=1)


def test_virtual_workers_reject_bad_args():
    from distributed_ml_pytorch_amd.runtime.trainer import TrainConfig
    from distributed_ml_pytorch_amd.runtime.virtual import VirtualWorkers

    with pytest.raises(ValueError):
        VirtualWorkers(TrainConfig(model="mlp", mode="sync", cuda=False), 2)
    with pytest.raises(ValueError):
        VirtualWorkers(TrainConfig(model="mlp", cuda=False), 0)


@pytest.mark.gpu
@pytest.mark.parametrize("model,graph,lr", [("mlp", False, 0.05), ("resnet18", True, 0.005)])
def test_virtual_workers_gpu_streams(model, graph, lr):
    k, steps = 3, 12
    out = _run(torch.device("cuda", 0), model, k=k, steps=steps, graph=graph, n_push=2,
               lr=lr)
    vw = out[0]
    assert len({s.cuda_stream for s in vw.streams}) == k
    _check(*out, k=k, steps=steps, n_push=2)
