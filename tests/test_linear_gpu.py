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


@pytest.mark.parametrize("M,K,N", [(1000, 768, 256), (394, 192, 128)])
def test_wgrad_fused_bias_every_config(M, K, N):
    """The bias gradient summed inside the weight-gradient kernel (ones-operand
    MFMA on the staged dY tiles), for every tile configuration the tuner may pick."""
    from distributed_ml_pytorch_amd.ops._ext import native
    from distributed_ml_pytorch_amd.ops.conv import _wgrad_candidates

    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    x4 = x.view(M, 1, 1, K).permute(0, 3, 1, 2)
    dy4 = dy.view(M, 1, 1, N).permute(0, 3, 1, 2)
    ref_w = dy.float().t() @ x.float()
    ref_b = dy.float().sum(0)
    for cfg in _wgrad_candidates(K, N):
        g = torch.zeros(N, K, device="cuda")
        b = torch.full((N,), 0.5, device="cuda")
        native().conv_wgrad(dy4, x4, g.view(N, K, 1, 1), 1, 0, cfg, b)
        assert float((g - ref_w).norm() / ref_w.norm()) < 1e-2, cfg
        torch.testing.assert_close(b, ref_b + 0.5, rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("B,C,H,P,D", [(4, 3, 224, 16, 768), (3, 3, 32, 4, 128)])
def test_patch_embed_gemm_matches_conv(B, C, H, P, D):
    """ViT patch embedding as one GEMM on gathered patch rows (channels-last
    arena weight as the [D, kh*kw*C] operand) vs an fp32 stride-P conv."""
    from distributed_ml_pytorch_amd.models.vit import PatchEmbed
    from distributed_ml_pytorch_amd.parallel.arena import FlatArena

    torch.manual_seed(0)
    pe = PatchEmbed(C, D, kernel_size=P, stride=P).cuda()
    arena = FlatArena(pe, device="cuda")
    x = torch.randn(B, C, H, H, device="cuda").to(torch.bfloat16)
    n = (H // P) ** 2
    c = torch.randn(B, n, D, device="cuda")
    y = pe(x)
    assert y.shape == (B, n, D) and y.dtype == torch.bfloat16
    (y.float() * c).sum().backward()
    w = pe.weight._dmp_w16.float().detach().requires_grad_(True)
    b = pe.bias._dmp_w16.float().detach().requires_grad_(True)
    yr = torch.nn.functional.conv2d(x.float(), w, b, stride=P).flatten(2).transpose(1, 2)
    (yr * c).sum().backward()
    rel = lambda a, r: float((a - r).norm() / (r.norm() + 1e-12))
    assert rel(y.float(), yr) < 1e-2
    assert rel(pe.weight.grad, w.grad) < 1e-2
    assert rel(pe.bias.grad, b.grad) < 1e-2
    assert pe.weight.grad.data_ptr() == arena.g32.data_ptr() + 4 * arena.slots[0].offset


@pytest.mark.parametrize("M,D,H", [(394, 768, 3072), (130, 64, 256)])
def test_fused_mlp_matches_fp32(M, D, H):
    """fc2(gelu(fc1(x))) as the fused native op (GELU in the fc1 forward
    epilogue, GELU' in the fc2 data-gradient epilogue) vs fp32 PyTorch on the
    same bf16 weights: output, input gradient, all four parameter gradients."""
    from distributed_ml_pytorch_amd.ops import layers as L
    from distributed_ml_pytorch_amd.ops.linear import mlp, mlp_ok
    from distributed_ml_pytorch_amd.parallel.arena import FlatArena

    torch.manual_seed(0)
    net = torch.nn.Sequential(L.Linear(D, H), L.Linear(H, D)).cuda()
    FlatArena(net, device="cuda")
    fc1, fc2 = net[0], net[1]
    x = torch.randn(M, D, device="cuda").to(torch.bfloat16).requires_grad_(True)
    assert mlp_ok(x, fc1, fc2)
    c = torch.randn(M, D, device="cuda")
    y = mlp(x, fc1, fc2)
    (y.float() * c).sum().backward()
    p = [t._dmp_w16.float().detach().requires_grad_(True)
         for t in (fc1.weight, fc1.bias, fc2.weight, fc2.bias)]
    xr = x.detach().float().requires_grad_(True)
    yr = torch.nn.functional.gelu(xr @ p[0].t() + p[1], approximate="tanh") @ p[2].t() + p[3]
    (yr * c).sum().backward()
    rel = lambda a, b: float((a.float() - b).norm() / (b.norm() + 1e-12))
    assert rel(y, yr) < 2e-2
    assert rel(x.grad, xr.grad) < 3e-2
    for t, r in zip((fc1.weight, fc1.bias, fc2.weight, fc2.bias), p):
        assert rel(t.grad, r.grad) < 3e-2


def test_linear_odd_head_native():
    """10-class head (N % 8 != 0) and 84-wide reduction run the any-shape native
    kernel in all three passes (LeNet fc3: 84 -> 10)."""
    from distributed_ml_pytorch_amd.ops import layers as L
    from distributed_ml_pytorch_amd.parallel.arena import FlatArena

    torch.manual_seed(0)
    lin = L.Linear(84, 10).cuda()
    FlatArena(lin, device="cuda")
    x = torch.randn(64, 84, device="cuda").to(torch.bfloat16).requires_grad_(True)
    c = torch.randn(64, 10, device="cuda")
    (lin(x).float() * c).sum().backward()
    w = lin.weight._dmp_w16.float().detach().requires_grad_(True)
    b = lin.bias._dmp_w16.float().detach().requires_grad_(True)
    xr = x.detach().float().requires_grad_(True)
    ((xr @ w.t() + b) * c).sum().backward()
    rel = lambda a, r: float((a.float() - r).norm() / (r.norm() + 1e-12))
    assert rel(lin.weight.grad, w.grad) < 1e-2
    assert rel(lin.bias.grad, b.grad) < 1e-2
    assert rel(x.grad, xr.grad) < 2e-2


@pytest.mark.parametrize("M,N,K,ldb", [(6, 75, 50176, 80), (16, 150, 6400, 152), (64, 27, 9000, 32),
                                       (10, 84, 4096, 88)])
@pytest.mark.parametrize("cfg,splits", [(4, 96), (9, 24), (-1, 196)])
def test_small_output_long_reduction_wgrad(M, N, K, ldb, cfg, splits):
    """Small-output / long-reduction weight gradient (LeNet's convs over
    B*OH*OW patch rows; the picks scripts/gemm_shape_sweep.py measures fastest:
    an MFMA tile split 24-128 ways over k with fp32 atomics, or the any-shape
    kernel): dW += dY^T X and dbias += colsum(dY) vs fp32, accumulating."""
    from distributed_ml_pytorch_amd.ops._ext import native

    torch.manual_seed(0)
    a = torch.randn(K, (M + 7) // 8 * 8, device="cuda").to(torch.bfloat16)[:, :M]
    bfull = torch.randn(K, ldb, device="cuda").to(torch.bfloat16)
    b = bfull[:, :N]
    c = torch.full((M, N), 0.25, device="cuda")
    db = torch.full((M,), -1.0, device="cuda")
    native().gemm(2, 3, cfg, a, b, c, None, None, None, db, splits, False, None, False)
    ref = a.float().t() @ b.float() + 0.25
    torch.testing.assert_close(c, ref, rtol=2e-3, atol=2e-3 * float(ref.abs().max()))
    torch.testing.assert_close(db, a.float().sum(0) - 1.0, rtol=2e-3, atol=1e-2)


@pytest.mark.parametrize("M,N,K", [(768, 256, 1000), (256, 384, 12608)])
def test_gemm_wgrad_every_config_split_slab(M, N, K):
    """Weight-gradient GEMM (dW[M][N] += dY^T X over K rows, + dbias) for every
    tile config of mode 2 -- including the 2-k-group 8-wave tile (cfg 9) --
    with and without split-K, atomics and slab reductions, vs fp32."""
    from distributed_ml_pytorch_amd.ops._ext import native

    torch.manual_seed(0)
    a = torch.randn(K, M, device="cuda").to(torch.bfloat16)
    b = torch.randn(K, N, device="cuda").to(torch.bfloat16)
    ref = a.float().t() @ b.float()
    refb = a.float().sum(0)
    cfgs = [c[0] for c in native().gemm_configs() if native().gemm_config_ok(2, c[0])]
    assert 9 in cfgs
    for cfg in cfgs:
        for splits, slab in ((1, False), (3, False), (3, True)):
            c = torch.full((M, N), 0.5, device="cuda")
            db = torch.zeros(M, device="cuda")
            native().gemm(2, 3, cfg, a, b, c, None, None, None, db, splits, False, None, slab)
            err = float((c - 0.5 - ref).norm() / ref.norm())
            assert err < 1e-2, (cfg, splits, slab, err)
            assert float((db - refb).norm() / refb.norm()) < 1e-2, (cfg, splits, slab)
