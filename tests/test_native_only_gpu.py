"""Every compute kernel of a training step is one of ours.

One eager ASGD training step (forward, backward, fused update, local PS push /
pull) of each model family under ``torch.profiler``, with the stock oracle mode
OFF (``ops._policy``: a GPU tensor that leaves native coverage raises instead
of running MIOpen / hipBLASLt / ATen).  Every device kernel must be a ``dmp::``
kernel; only copy engine work (the input batch moved into the step's buffers)
is allowed besides.  Also: ``--dtype fp32`` on the GPU is refused outside the
oracle mode, and an op outside native coverage raises.
"""
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.strict_native]

# (vit_tiny's head dim 16 is outside the fused attention kernel: on the GPU it runs
# only in the oracle mode, which test_op_outside_native_coverage_raises covers)
MODELS = [("resnet18", 16), ("resnet50", 4), ("vit_b16", 2), ("alexnet", 16), ("lenet", 16),
          ("mlp", 16)]


def _is_copy(name: str) -> bool:
    return name.startswith(("__amd_rocclr_copyBuffer", "Memcpy", "memcpy"))


@pytest.mark.parametrize("model,batch", MODELS)
def test_training_step_runs_only_native_kernels(model, batch):
    from torch.profiler import ProfilerActivity, profile

    from distributed_ml_pytorch_amd.runtime.dist import DistInfo
    from distributed_ml_pytorch_amd.runtime.trainer import TrainConfig, Worker

    info = DistInfo(device=torch.device("cuda", 0))
    cfg = TrainConfig(model=model, batch_size=batch, mode="asgd", ps="local", n_push=1,
                      n_pull=1, lr=0.01, evaluate=False, verbose=False)
    w = Worker(cfg, info)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(batch, *w.input_shape, generator=g)
    y = torch.randint(0, w.num_classes, (batch,), generator=g)
    x, y = w.prepare(x, y)
    w.train_step(x, y)                    # first step: per-shape kernel picks (all native)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        loss, _ = w.train_step(x, y)
        torch.cuda.synchronize()
    w.finish()
    names = [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
    assert names, "profiler recorded no device work"
    foreign = sorted({n for n in names if "dmp::" not in n and not _is_copy(n)})
    assert not foreign, f"{model}: non-native device kernels in a training step: {foreign}"
    assert sum("dmp::" in n for n in names) >= 5, names
    lv = float(loss.float().item())
    assert lv == lv and lv > 0


def test_fp32_gpu_training_is_refused():
    from distributed_ml_pytorch_amd.runtime.dist import DistInfo
    from distributed_ml_pytorch_amd.runtime.trainer import TrainConfig, Worker

    cfg = TrainConfig(model="lenet", batch_size=8, mode="asgd", ps="local", dtype="fp32",
                      evaluate=False, verbose=False)
    with pytest.raises(ValueError, match="stock"):
        Worker(cfg, DistInfo(device=torch.device("cuda", 0)))


def test_op_outside_native_coverage_raises():
    from distributed_ml_pytorch_amd.ops import functional as DF
    from distributed_ml_pytorch_amd.ops._policy import (NativeCoverageError, stock_allowed,
                                                        stock_log)

    q = torch.randn(2, 4, 16, 32, device="cuda", dtype=torch.bfloat16)   # head dim 32
    with pytest.raises(NativeCoverageError, match="attention"):
        DF.attention(q, q, q)
    x = torch.randn(4, 8, device="cuda")                                  # fp32
    with pytest.raises(NativeCoverageError, match="relu"):
        DF.relu(x)
    with stock_allowed(True):             # the explicit oracle mode: runs, and is logged
        DF.relu(x)
    assert any(op == "relu" for op, _ in stock_log())
