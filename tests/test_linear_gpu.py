"""Arena linear (bf16 GEMMs, fp32 weight grad accumulated in place) vs fp32 PyTorch."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,K,N,bias", [(256, 512, 10, True), (96, 768, 3072, True),
                                        (394, 3072, 768, True),
                                        (33, 120, 84, False)])
def test_arena_linear_grads(M, K, N, bias):
    from distributed_ml_pytorch_amd.ops import layers as L
    from distributed_ml_pytorch_amd.parallel.arena import FlatArena

    torch.manual_seed(0)
    lin = L.Linear(K, N, bias=bias).cuda()
    arena = FlatArena(lin, device="cuda")
    ready = []
    arena.set_grad_ready_callback(lambda i: ready.append(i))
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16).requires_grad_(True)
    c = torch.randn(M, N, device="cuda")
    for rep in (1, 2):
        y = lin(x)
        assert y.dtype == torch.bfloat16
        (y.float() * c).sum().backward()
    # fp32 reference on the same bf16 operands
    w16 = lin.weight._dmp_w16.float().detach().requires_grad_(True)
    xr = x.detach().float().requires_grad_(True)
    yr = xr @ w16.t()
    if bias:
        b16 = lin.bias._dmp_w16.float().detach().requires_grad_(True)
        yr = yr + b16
    (yr * c).sum().backward()
    rel = lambda a, b: float((a - b).norm() / (b.norm() + 1e-12))
    assert rel(lin.weight.grad, 2 * w16.grad) < 1e-2
    assert lin.weight.grad.data_ptr() == arena.g32.data_ptr() + 4 * arena.slots[0].offset
    if bias:
        assert rel(lin.bias.grad, 2 * b16.grad) < 1e-2
    assert rel(x.grad.float(), 2 * xr.grad) < 2e-2
    assert 0 in ready
