"""Inference (``torch.no_grad()``) paths on the native kernels, and the ViT token
assembly kernel pair.

The reference evaluates the whole 10k-image test set every ``log_interval``
iterations (/root/reference/example/main.py:83-84,110-125): that forward runs
under no_grad, so every Linear / MLP / patch-embedding GEMM and the token
assembly must take the native path there too (not hipBLASLt / MIOpen / ATen).
Oracles: the training-mode forward on the same kernels (bit-identical) and a
plain fp32 PyTorch formulation.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _model(name, **kw):
    from distributed_ml_pytorch_amd.models import build_model
    from distributed_ml_pytorch_amd.parallel.arena import attach_arena

    torch.manual_seed(0)
    m, shape, nc = build_model(name, **kw)
    m = m.cuda()
    attach_arena(m, shadow_dtype=torch.bfloat16, channels_last=True)
    return m, shape, nc


@pytest.mark.parametrize("name,batch", [("vit_tiny", 6), ("alexnet", 64), ("lenet", 32),
                                        ("mlp", 16)])
def test_no_grad_forward_matches_grad_forward(name, batch):
    """Eval forward under no_grad == the same forward with autograd recording
    (same native kernels, no autograd nodes, no saved tensors)."""
    from distributed_ml_pytorch_amd.ops import linear as LIN

    m, shape, _ = _model(name)
    m.eval()
    x = torch.randn(batch, *shape, device="cuda").to(torch.bfloat16)
    if x.dim() == 4:
        x = x.contiguous(memory_format=torch.channels_last)
    y_grad = m(x)
    assert y_grad.requires_grad
    calls = []
    orig = LIN._infer_linear
    LIN._infer_linear = lambda *a, **k: calls.append(1) or orig(*a, **k)
    try:
        with torch.no_grad():
            y = m(x)
    finally:
        LIN._infer_linear = orig
    assert not y.requires_grad
    assert calls, "no-grad forward did not take the native inference GEMM"
    torch.testing.assert_close(y, y_grad.detach(), rtol=0, atol=0)


def test_vit_embed_matches_torch():
    from distributed_ml_pytorch_amd.ops import functional as DF

    torch.manual_seed(1)
    B, N, D = 5, 196, 768
    tok = torch.randn(B, N, D, device="cuda").to(torch.bfloat16).requires_grad_(True)
    cls = torch.nn.Parameter(torch.randn(1, 1, D, device="cuda"))
    pos = torch.nn.Parameter(torch.randn(1, N + 1, D, device="cuda"))
    h = DF.vit_embed(tok, cls, pos)
    g = torch.randn(B, N + 1, D, device="cuda").to(torch.bfloat16)
    h.backward(g)
    tr = tok.detach().float().requires_grad_(True)
    cr = cls.detach().to(torch.bfloat16).float().requires_grad_(True)
    pr = pos.detach().to(torch.bfloat16).float().requires_grad_(True)
    hr = torch.cat([cr.expand(B, -1, -1), tr], 1) + pr
    hr.backward(g.float())
    torch.testing.assert_close(h.float(), hr, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(tok.grad.float(), tr.grad)
    torch.testing.assert_close(cls.grad, cr.grad, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(pos.grad, pr.grad, rtol=1e-5, atol=1e-4)


def test_vit_embed_accumulates_into_arena():
    """Arena-backed cls / pos: the batch sums land in the flat grad buffer."""
    m, shape, _ = _model("vit_tiny")
    m.train()
    x = torch.randn(4, *shape, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    for p in m.parameters():
        p.grad.zero_()
    m(x).float().sum().backward()
    assert float(m.pos_embed.grad.abs().sum()) > 0
    assert float(m.cls_token.grad.abs().sum()) > 0
    # row 0 of the position gradient and the class-token gradient are the same sum
    torch.testing.assert_close(m.pos_embed.grad[0, 0], m.cls_token.grad[0, 0])
