"""Native MFMA GEMM (csrc/gemm.hip) vs a plain fp32 PyTorch oracle: every mode
(fwd / dgrad / wgrad), every fused epilogue and every tile config, on shapes
with tails in every dimension and asymmetric operands (a transposed store or a
swapped operand map cannot pass)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


def _gelu(x):
    return torch.nn.functional.gelu(x, approximate="tanh")


def _cfgs(mode):
    from distributed_ml_pytorch_amd.ops._ext import native

    return [-1] + [c[0] for c in native().gemm_configs() if native().gemm_config_ok(mode, c[0])]


SHAPES = [(300, 256, 264), (64, 768, 128), (1000, 192, 520), (257, 136, 72)]


@pytest.mark.parametrize("M,K,N", SHAPES)
@pytest.mark.parametrize("epi", ["plain", "bias_addend", "gelu"])
def test_gemm_fwd(M, K, N, epi):
    from distributed_ml_pytorch_amd.ops._ext import native

    torch.manual_seed(1)
    dev = "cuda"
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    # asymmetric, row-dependent weights
    w = (torch.randn(N, K, device=dev) + 0.01 * torch.arange(N, device=dev)[:, None]).to(
        torch.bfloat16)
    b = torch.randn(N, device=dev).to(torch.bfloat16)
    r = torch.randn(M, N, device=dev).to(torch.bfloat16)
    ref = x.float() @ w.float().t()
    for cfg in _cfgs(0):
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        if epi == "plain":
            native().gemm(0, 0, cfg, x, w, y)
            assert _rel(y, ref) < 1e-2, cfg
        elif epi == "bias_addend":
            native().gemm(0, 0, cfg, x, w, y, bias=b, aux=r)
            assert _rel(y, ref + b.float() + r.float()) < 1e-2, cfg
        else:
            g = torch.empty_like(y)
            native().gemm(0, 1, cfg, x, w, y, c2=g, bias=b)
            h = ref + b.float()
            assert _rel(y, h) < 1e-2, cfg
            assert _rel(g, _gelu(y.float())) < 1e-2, cfg


@pytest.mark.parametrize("M,K,N", SHAPES)
@pytest.mark.parametrize("dgelu", [False, True])
def test_gemm_dgrad(M, K, N, dgelu):
    """dX[M, K] = dY[M, N] @ W[N, K] (W read k-strided through transposed LDS reads)."""
    from distributed_ml_pytorch_amd.ops._ext import native

    torch.manual_seed(2)
    dev = "cuda"
    dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) + 0.01 * torch.arange(K, device=dev)[None, :]).to(
        torch.bfloat16)
    h = torch.randn(M, K, device=dev).to(torch.bfloat16)
    ref = dy.float() @ w.float()
    if dgelu:
        hr = h.float().requires_grad_(True)
        _gelu(hr).backward(ref)
        ref = hr.grad
    for cfg in _cfgs(1):
        dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        native().gemm(1, 2 if dgelu else 0, cfg, dy, w, dx, aux=h if dgelu else None)
        assert _rel(dx, ref) < 1.5e-2, cfg


@pytest.mark.parametrize("M,K,N", SHAPES)
@pytest.mark.parametrize("splits,slab", [(1, False), (3, False), (3, True)])
def test_gemm_wgrad(M, K, N, splits, slab):
    """gW[N, K] += dY^T X, gb[N] += colsum(dY), fp32 accumulate (split-K with atomics,
    or through a plain-store partial slab + reduce pass)."""
    from distributed_ml_pytorch_amd.ops._ext import native

    torch.manual_seed(3)
    dev = "cuda"
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    dy = (torch.randn(M, N, device=dev) + 0.02 * torch.arange(N, device=dev)[None, :]).to(
        torch.bfloat16)
    ref_w = dy.float().t() @ x.float()
    ref_b = dy.float().sum(0)
    # split-K: both block -> (tile, k-range) deals (GemmArgs::xcd_k)
    try:
        for xcd_k in ((0, 1) if splits > 1 else (1,)):
            native().gemm_set_xcd_k(xcd_k)
            for cfg in _cfgs(2):
                g = torch.full((N, K), 0.25, device=dev)
                gb = torch.full((N,), -0.5, device=dev)
                native().gemm(2, 3, cfg, dy, x, g, dbias=gb, splits=splits, slab=slab)
                assert _rel(g - 0.25, ref_w) < 2e-3, (cfg, xcd_k)
                assert _rel(gb + 0.5, ref_b) < 2e-3, (cfg, xcd_k)
    finally:
        native().gemm_set_xcd_k(1)


def test_gemm_strided_operands():
    """Row strides wider than the row (column slices of a bigger buffer)."""
    from distributed_ml_pytorch_amd.ops._ext import native

    torch.manual_seed(4)
    big = torch.randn(200, 520, device="cuda").to(torch.bfloat16)
    x = big[:, 8:264]                      # [200, 256], ld 520
    w = torch.randn(136, 256, device="cuda").to(torch.bfloat16)
    ref = x.float() @ w.float().t()
    for cfg in _cfgs(0):
        y = torch.empty(200, 136, device="cuda", dtype=torch.bfloat16)
        native().gemm(0, 0, cfg, x, w, y)
        assert _rel(y, ref) < 1e-2, cfg


def test_gemm_rejects_bad_shapes():
    from distributed_ml_pytorch_amd.ops._ext import native

    x = torch.randn(64, 84, device="cuda").to(torch.bfloat16)
    w = torch.randn(10, 84, device="cuda").to(torch.bfloat16)
    y = torch.empty(64, 10, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        native().gemm(0, 0, 0, x, w, y)      # K % 8 != 0 on the MFMA path
    dy = torch.randn(64, 136, device="cuda").to(torch.bfloat16)
    w2 = torch.randn(136, 192, device="cuda").to(torch.bfloat16)
    dx = torch.empty(64, 192, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        native().gemm(1, 0, 6, dy, w2, dx)   # 192-wide tile on a k-strided operand
    native().gemm(0, 0, -1, x, w, y)         # the any-shape kernel takes it
    assert _rel(y, x.float() @ w.float().t()) < 1e-2


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_gemm_persistent_many_tiles(mode):
    """More tiles than resident blocks: each persistent block walks several tiles
    and its DMA ring runs across tile boundaries (short K: 2-4 k-tiles/tile)."""
    from distributed_ml_pytorch_amd.ops._ext import native

    torch.manual_seed(5)
    dev = "cuda"
    if mode == 2:
        T, K, N = 192, 8192, 2304                 # dW [2304, 8192]: 288 tiles of 256x256
        x = torch.randn(T, K, device=dev).to(torch.bfloat16)
        dy = torch.randn(T, N, device=dev).to(torch.bfloat16)
        ref = dy.float().t() @ x.float()
        for cfg in _cfgs(2)[1:]:
            g = torch.zeros(N, K, device=dev)
            native().gemm(2, 3, cfg, dy, x, g)
            assert _rel(g, ref) < 2e-3, cfg
        return
    M, K, N = 12608, 128, 2304
    a = torch.randn(M, K if mode == 0 else N, device=dev).to(torch.bfloat16)
    w = torch.randn(N, K, device=dev).to(torch.bfloat16)
    b = torch.randn(N, device=dev).to(torch.bfloat16)
    if mode == 0:
        ref = a.float() @ w.float().t() + b.float()
    else:
        ref = a.float() @ w.float()
    for cfg in _cfgs(mode)[1:]:
        out = torch.empty(M, N if mode == 0 else K, device=dev, dtype=torch.bfloat16)
        if mode == 0:
            native().gemm(0, 0, cfg, a, w, out, bias=b)
        else:
            native().gemm(1, 0, cfg, a, w, out)
        assert _rel(out, ref) < 1e-2, cfg


def _sk_shape(cfg, K, N, want=2):
    """An M whose tile count leaves a last partial round that the remainder
    split-K plan of ``cfg`` actually splits (depends on the CU count)."""
    from distributed_ml_pytorch_amd.ops._ext import native

    info = {c[0]: c for c in native().gemm_configs()}[cfg]
    bm = info[1]
    for tiles_m in range(8, 400):
        M = tiles_m * bm - 37          # a row tail in the last M tile too
        if native().gemm_sk_pieces(cfg, M, N, K, want) > 0:
            return M
    return None


@pytest.mark.parametrize("mode,epi", [(0, "bias_addend"), (0, "gelu"), (1, "plain"),
                                      (1, "dgelu"), (1, "drelu")])
def test_gemm_remainder_split_k(mode, epi):
    """fwd / dgrad with the last partial round's tiles split along K (csrc/gemm.hip
    GemmArgs sk_*): every piece publishes fp32 partials, the last arriver adds them
    and runs the epilogue -- against fp32 PyTorch and against the unsplit launch.
    The bias / addend / GELU epilogues must be applied exactly once."""
    from distributed_ml_pytorch_amd.ops._ext import native

    torch.manual_seed(5)
    dev = "cuda"
    K, N = 520, 512
    tried = 0
    for cfg in [c for c in _cfgs(mode) if c >= 0]:
        for want in (2, 4):
            M = _sk_shape(cfg, K, N, want)
            if M is None:
                continue
            tried += 1
            b = torch.randn(N, device=dev).to(torch.bfloat16)
            if mode == 0:
                x = torch.randn(M, K, device=dev).to(torch.bfloat16)
                w = (torch.randn(N, K, device=dev) + 0.01 * torch.arange(N, device=dev)[:, None]
                     ).to(torch.bfloat16)
                r = torch.randn(M, N, device=dev).to(torch.bfloat16)
                ref = x.float() @ w.float().t() + b.float()
                y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                y1 = torch.empty_like(y)
                if epi == "bias_addend":
                    native().gemm(0, 0, cfg, x, w, y, bias=b, aux=r, splits=want)
                    native().gemm(0, 0, cfg, x, w, y1, bias=b, aux=r)
                    assert _rel(y, ref + r.float()) < 1e-2, (cfg, want)
                else:
                    g = torch.empty_like(y)
                    native().gemm(0, 1, cfg, x, w, y, c2=g, bias=b, splits=want)
                    native().gemm(0, 1, cfg, x, w, y1, c2=torch.empty_like(y), bias=b)
                    assert _rel(y, ref) < 1e-2 and _rel(g, _gelu(y.float())) < 1e-2, (cfg, want)
                assert _rel(y, y1) < 4e-3, (cfg, want)
            else:
                dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
                w = (torch.randn(N, K, device=dev) + 0.01 * torch.arange(K, device=dev)[None, :]
                     ).to(torch.bfloat16)
                h = torch.randn(M, K, device=dev).to(torch.bfloat16)
                ref = dy.float() @ w.float()
                e, aux = 0, None
                if epi == "dgelu":
                    hr = h.float().requires_grad_(True)
                    _gelu(hr).backward(ref)
                    ref, e, aux = hr.grad, 2, h
                elif epi == "drelu":
                    ref, e, aux = ref * (h.float() > 0), 4, h
                dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
                dx1 = torch.empty_like(dx)
                native().gemm(1, e, cfg, dy, w, dx, aux=aux, splits=want)
                native().gemm(1, e, cfg, dy, w, dx1, aux=aux)
                assert _rel(dx, ref) < 1.5e-2, (cfg, want)
                assert _rel(dx, dx1) < 4e-3, (cfg, want)
    assert tried > 0


def test_gemm_store_addend_bitmask():
    """Store epilogue with a deferred ReLU bit mask on its addend (GemmArgs::auxmask,
    the residual gradient of a Bottleneck's identity shortcut) == the same GEMM with
    the addend masked beforehand, bitwise, on every MFMA config; the wrapper
    materialises the mask for the library / fallback picks."""
    from distributed_ml_pytorch_amd.ops._ext import native
    from distributed_ml_pytorch_amd.ops.functional import apply_bitmask_rows

    nat = native()
    torch.manual_seed(5)
    M, N, K = 1000, 256, 192
    dy = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(K, N, device="cuda") / K ** 0.5).to(torch.bfloat16)
    aux = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    mask = torch.randint(0, 256, (M * N // 8,), device="cuda", dtype=torch.uint8)
    masked = apply_bitmask_rows(aux, mask)
    ref32 = dy.float() @ w.float() + masked.float()
    ran = 0
    for c in [c[0] for c in nat.gemm_configs()]:
        if not nat.gemm_config_ok(1, c):
            continue
        ran += 1
        ref = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        got = torch.empty_like(ref)
        nat.gemm(1, 0, c, dy, w, ref, aux=masked)
        nat.gemm(1, 0, c, dy, w, got, aux=aux, auxmask=mask)
        assert torch.equal(got, ref), c
        assert (got.float() - ref32).norm() / ref32.norm() < 1e-2
    assert ran > 0
