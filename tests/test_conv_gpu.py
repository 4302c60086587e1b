"""Native NHWC implicit-GEMM conv (fwd / dgrad / wgrad / fused BN partials) vs fp32 PyTorch."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
CL = torch.channels_last

SHAPES = [
    # B, CI, H, W, CO, k, stride, pad
    (4, 64, 32, 32, 64, 3, 1, 1),
    (2, 64, 16, 16, 128, 3, 2, 1),
    (2, 64, 16, 16, 128, 1, 2, 0),
    (3, 128, 8, 8, 256, 3, 1, 1),
    (2, 256, 8, 8, 512, 3, 2, 1),
    (2, 192, 4, 4, 384, 3, 1, 1),      # AlexNet conv3 (CI=192: BK=64 tiles)
    (2, 64, 5, 7, 64, 3, 1, 1),        # odd spatial, M not a tile multiple
    (1, 512, 4, 4, 512, 3, 1, 1),
]


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


@pytest.mark.parametrize("B,CI,H,W,CO,k,st,pd", SHAPES)
def test_conv_fwd_dgrad_wgrad(B, CI, H, W, CO, k, st, pd):
    from distributed_ml_pytorch_amd.ops._ext import native

    nat = native()
    torch.manual_seed(0)
    x = torch.randn(B, CI, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(CO, CI, k, k, device="cuda") / (CI * k * k) ** 0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=CL)
    y, part, G = nat.conv_fwd(x, w, st, pd, True)
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    yr = F.conv2d(xr, wr, None, st, pd)
    assert y.shape == yr.shape and y.is_contiguous(memory_format=CL)
    assert _rel(y, yr) < 1e-2
    # fused BN partial sums == per-channel sums of the (bf16-rounded) output
    C = CO
    G = int(G)
    ps = part[:2 * G * C].view(2, G, C).sum(1)
    yf = y.float()
    torch.testing.assert_close(ps[0], yf.sum(dim=(0, 2, 3)), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(ps[1], (yf * yf).sum(dim=(0, 2, 3)), rtol=1e-3, atol=1e-2)
    # backward
    dy = torch.randn_like(yr).to(torch.bfloat16).contiguous(memory_format=CL)
    yr.backward(dy.float())
    dx = nat.conv_dgrad(dy, w, H, W, st, pd)
    assert dx.shape == x.shape
    assert _rel(dx, xr.grad) < 1e-2
    dw = torch.zeros(CO, CI, k, k, device="cuda").contiguous(memory_format=CL)
    nat.conv_wgrad(dy, x, dw, st, pd)
    assert _rel(dw, wr.grad) < 1e-2
    # accumulation semantics (fp32 atomics add into the existing grad)
    nat.conv_wgrad(dy, x, dw, st, pd)
    assert _rel(dw, 2 * wr.grad) < 1e-2


@pytest.mark.parametrize("shape", [(2, 64, 9, 11, 128, 3, 2, 1), (2, 128, 8, 8, 64, 1, 1, 0)])
def test_every_tile_config(shape):
    """The tuner may pick any compiled tile: each must be exact on odd shapes."""
    from distributed_ml_pytorch_amd.ops._ext import native

    nat = native()
    B, CI, H, W, CO, k, st, pd = shape
    x = torch.randn(B, CI, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(CO, CI, k, k, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=CL)
    yr = F.conv2d(x.float(), w.float(), None, st, pd)
    dy = torch.randn_like(yr).to(torch.bfloat16).contiguous(memory_format=CL)
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    F.conv2d(xr, wr, None, st, pd).backward(dy.float())
    for cfg in [c[0] for c in nat.conv_configs()]:
        y, part, G = nat.conv_fwd(x, w, st, pd, True, cfg)
        assert _rel(y, yr) < 1e-2, cfg
        ps = part[:2 * int(G) * CO].view(2, int(G), CO).sum(1)
        torch.testing.assert_close(ps[0], y.float().sum(dim=(0, 2, 3)), rtol=1e-3, atol=1e-2)
        dx = nat.conv_dgrad(dy, w, H, W, st, pd, cfg)
        assert _rel(dx, xr.grad) < 1e-2, cfg
    from distributed_ml_pytorch_amd.ops.conv import _wgrad_candidates

    for cfg in _wgrad_candidates(CI * k * k, CO):
        dw = torch.zeros(CO, CI, k, k, device="cuda").contiguous(memory_format=CL)
        nat.conv_wgrad(dy, x, dw, st, pd, cfg)
        assert _rel(dw, wr.grad) < 1e-2, cfg


HALO_SHAPES = [
    # B, C, H, W, CO: every ResNet-18 CIFAR 3x3 stride-1 geometry, partial last tile
    (4, 64, 32, 32, 64),
    (3, 128, 16, 16, 128),
    (5, 256, 8, 8, 256),
    (9, 512, 4, 4, 512),
    (2, 64, 8, 8, 128),
    (2, 64, 56, 56, 64),      # ImageNet ResNet stage 1: 7x16-pixel row tiles (224 / 112 / 448)
    (3, 128, 28, 28, 128),    # stage 2: 4 rows of 28 (no halo wgrad tile fits 28-pixel rows)
    (3, 256, 14, 14, 256),    # stage 3: padded whole-image tiles (1 image in 224 rows, 2 in 448)
    (5, 512, 7, 7, 512),      # stage 4: 2 / 4 / 5 / 9 / 10 images in 112 / 224 / 256 / 448 / 512 rows
]


@pytest.mark.parametrize("B,C,H,W,CO", HALO_SHAPES)
def test_halo_conv_configs(B, C, H, W, CO):
    """3x3/stride-1 halo-tile kernels, every applicable config: forward (+BN partial
    sums), the mirrored-tap data gradient (+ residual addend) and the tap-row
    weight gradient (fp32 accumulate) vs fp32."""
    from distributed_ml_pytorch_amd.ops._ext import native

    nat = native()
    torch.manual_seed(0)
    x = torch.randn(B, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(CO, C, 3, 3, device="cuda") / (C * 9) ** 0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=CL)
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    yr = F.conv2d(xr, wr, None, 1, 1)
    dy = torch.randn_like(yr).to(torch.bfloat16).contiguous(memory_format=CL)
    yr.backward(dy.float())
    add = torch.randn_like(x)
    cfgs = list(nat.conv_halo_configs(H, W, C, 3, 3, 1, 1))
    assert cfgs, "no halo config applies"
    for cfg in cfgs:
        y, part, G = nat.conv_fwd(x, w, 1, 1, True, cfg)
        assert _rel(y, yr) < 1e-2, cfg
        ps = part[:2 * int(G) * CO].view(2, int(G), CO).sum(1)
        yf = y.float()
        torch.testing.assert_close(ps[0], yf.sum(dim=(0, 2, 3)), rtol=1e-3, atol=1e-2)
        torch.testing.assert_close(ps[1], (yf * yf).sum(dim=(0, 2, 3)), rtol=1e-3, atol=1e-2)
    for cfg in list(nat.conv_halo_configs(H, W, CO, 3, 3, 1, 1)):
        dx = nat.conv_dgrad(dy, w, H, W, 1, 1, cfg)
        assert _rel(dx, xr.grad) < 1e-2, cfg
        dxa = nat.conv_dgrad(dy, w, H, W, 1, 1, cfg, None, add)
        assert _rel(dxa, xr.grad + add.float()) < 1e-2, cfg
    wcfgs = list(nat.conv_wgrad_halo_configs(B, H, W, C, CO, 3, 3, 1, 1))
    assert wcfgs or W in (28, 14, 7), "no halo wgrad config applies"
    for cfg in wcfgs:
        dw = torch.zeros(CO, C, 3, 3, device="cuda").contiguous(memory_format=CL)
        nat.conv_wgrad(dy, x, dw, 1, 1, cfg)
        assert _rel(dw, wr.grad) < 1e-2, cfg
        nat.conv_wgrad(dy, x, dw, 1, 1, cfg)       # accumulates (atomic or owned tiles)
        assert _rel(dw, 2 * wr.grad) < 1e-2, cfg


@pytest.mark.parametrize("B,CI,H,CO,k,st,pd", [(3, 64, 14, 256, 1, 1, 0), (2, 256, 7, 64, 1, 1, 0),
                                                (2, 64, 9, 128, 3, 1, 1), (3, 64, 8, 64, 3, 2, 1)])
def test_igemm_row_epilogue_configs(B, CI, H, CO, k, st, pd):
    """Implicit-GEMM forward tiles with the row-staged epilogue (cfg ids 24-27):
    output + BN partial sums, and the bias / addend / ReLU inference epilogue, vs fp32."""
    from distributed_ml_pytorch_amd.ops._ext import native

    nat = native()
    torch.manual_seed(0)
    x = torch.randn(B, CI, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(CO, CI, k, k, device="cuda") / (CI * k * k) ** 0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=CL)
    yr = F.conv2d(x.float(), w.float(), None, st, pd)
    bias = torch.randn(CO, device="cuda")
    add = torch.randn_like(yr).to(torch.bfloat16).contiguous(memory_format=CL)
    for cfg in (24, 25, 26, 27):
        y, part, G = nat.conv_fwd(x, w, st, pd, True, cfg)
        assert _rel(y, yr) < 1e-2, cfg
        ps = part[:2 * int(G) * CO].view(2, int(G), CO).sum(1)
        yf = y.float()
        torch.testing.assert_close(ps[0], yf.sum(dim=(0, 2, 3)), rtol=1e-3, atol=1e-2)
        torch.testing.assert_close(ps[1], (yf * yf).sum(dim=(0, 2, 3)), rtol=1e-3, atol=1e-2)
        y2, _, _ = nat.conv_fwd(x, w, st, pd, False, cfg, None, bias, True, add)
        ref = torch.relu(yr + bias.view(1, -1, 1, 1) + add.float())
        assert _rel(y2, ref) < 1e-2, cfg
        dx = nat.conv_dgrad(add, w, H, H, st, pd, cfg)      # as a data-gradient tile: plain epilogue
        xr = x.float().requires_grad_(True)
        F.conv2d(xr, w.float(), None, st, pd).backward(add.float())
        assert _rel(dx, xr.grad) < 1e-2, cfg


@pytest.mark.parametrize("B,C,H,CO", [
    (3, 64, 32, 128), (5, 128, 16, 256), (9, 256, 8, 512),      # ResNet-18 stride-2 3x3 convs
    (2, 128, 56, 128),                                          # ResNet-50 (v1.5) stage-2 stride-2 3x3
])
def test_halo_wgrad_stride2(B, C, H, CO):
    """3x3 / stride-2 halo weight gradient (conv_wgrad_halo_kernel<S2>), every
    applicable config (atomic and slab split-K) vs fp32 autograd, accumulating."""
    from distributed_ml_pytorch_amd.ops._ext import native

    nat = native()
    torch.manual_seed(0)
    x = torch.randn(B, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    xr = x.float()
    wr = torch.zeros(CO, C, 3, 3, device="cuda", requires_grad=True)
    yr = F.conv2d(xr, wr, None, 2, 1)
    dy = torch.randn_like(yr).to(torch.bfloat16).contiguous(memory_format=CL)
    yr.backward(dy.float())
    cfgs = list(nat.conv_wgrad_halo_configs(B, H, H, C, CO, 3, 3, 2, 1))
    assert cfgs, "no stride-2 halo wgrad config applies"
    for cfg in cfgs:
        dw = torch.zeros(CO, C, 3, 3, device="cuda").contiguous(memory_format=CL)
        nat.conv_wgrad(dy, x, dw, 2, 1, cfg)
        assert _rel(dw, wr.grad) < 1e-2, cfg
        nat.conv_wgrad(dy, x, dw, 2, 1, cfg)
        assert _rel(dw, 2 * wr.grad) < 1e-2, cfg


@pytest.mark.parametrize("B,H", [(3, 32), (1, 32), (5, 16), (7, 8)])
@pytest.mark.parametrize("with_add", [False, True])
def test_halo64p_addend_matrix(B, H, with_add):
    """The persistent 64-channel kernels (ids 115-117) load their residual addend
    with inline-asm loads whose completion the epilogue counts by hand (vmcnt):
    every config x {no addend, full addend} x {odd batch, B = 1, whole-row and
    whole-image tiles, tile counts that do not fill the grid evenly}, forward
    (+fp32 bias, ReLU: the inference-time BN fold) and data gradient vs fp32.
    (ImageNet 56 x 56 rows are not a divisor of the 256 / 128-pixel tiles: no
    persistent config is offered there -- checked below -- and those layers run
    the 224-pixel halo tiles of test_halo_conv_configs.)"""
    from distributed_ml_pytorch_amd.ops._ext import native

    nat = native()
    torch.manual_seed(1)
    C = 64
    x = torch.randn(B, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(C, C, 3, 3, device="cuda") / (C * 9) ** 0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=CL)
    bias = torch.randn(C, device="cuda") * 0.1
    add = torch.randn_like(x) if with_add else None
    xr = x.float().requires_grad_(True)
    yr = F.conv2d(xr, w.float(), None, 1, 1)
    dy = torch.randn_like(yr).to(torch.bfloat16).contiguous(memory_format=CL)
    yr.backward(dy.float())
    ref_f = torch.relu(yr.detach() + bias.view(1, -1, 1, 1) + (add.float() if with_add else 0))
    ref_d = xr.grad + (add.float() if with_add else 0)
    ran = 0
    for cfg in (115, 116, 117):
        if cfg not in list(nat.conv_halo_configs(H, H, C, 3, 3, 1, 1)):
            continue
        ran += 1
        y, _, _ = nat.conv_fwd(x, w, 1, 1, False, cfg, None, bias, True, add)
        assert torch.isfinite(y.float()).all(), cfg
        assert _rel(y, ref_f) < 1e-2, (cfg, _rel(y, ref_f))
        dx = nat.conv_dgrad(dy, w, H, H, 1, 1, cfg, None, add)
        assert torch.isfinite(dx.float()).all(), cfg
        assert _rel(dx, ref_d) < 1e-2, (cfg, _rel(dx, ref_d))
    assert ran > 0
    assert not set(nat.conv_halo_configs(56, 56, C, 3, 3, 1, 1)) & {115, 116, 117}


@pytest.mark.parametrize("cfg_kind", ["halo", "igemm"])
def test_conv_fwd_bias_addend_relu_epilogue(cfg_kind):
    """Forward epilogue of the inference-time BN fold on the non-persistent tiles:
    relu(conv(x) + bias + addend), every applicable config."""
    from distributed_ml_pytorch_amd.ops._ext import native

    nat = native()
    torch.manual_seed(2)
    B, C, H, CO = 3, 128, 16, 128
    x = torch.randn(B, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(CO, C, 3, 3, device="cuda") / (C * 9) ** 0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=CL)
    bias = torch.randn(CO, device="cuda") * 0.1
    add = torch.randn(B, CO, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    ref = torch.relu(F.conv2d(x.float(), w.float(), None, 1, 1) + bias.view(1, -1, 1, 1)
                     + add.float())
    from distributed_ml_pytorch_amd.ops.conv import _igemm_candidates

    cfgs = list(nat.conv_halo_configs(H, H, C, 3, 3, 1, 1)) if cfg_kind == "halo" else \
        _igemm_candidates(CO)
    for cfg in cfgs:
        y, _, _ = nat.conv_fwd(x, w, 1, 1, False, cfg, None, bias, True, add)
        assert _rel(y, ref) < 1e-2, (cfg, _rel(y, ref))


@pytest.mark.parametrize("model,shape", [("resnet18", (3, 32, 32)), ("resnet50", (3, 64, 64)),
                                         ("resnet50", (3, 224, 224))])   # 224: the 7x7 stem kernel
def test_eval_bn_fold_matches_unfolded_eval(model, shape):
    """Eval forward with every BatchNorm folded into its conv (ops/eval_fold.py)
    == the regular eval forward (running-statistics BN passes), after a few
    training steps moved the running statistics away from their init."""
    import os

    from distributed_ml_pytorch_amd.models import build_model
    from distributed_ml_pytorch_amd.ops import eval_fold
    from distributed_ml_pytorch_amd.ops.functional import softmax_cross_entropy
    from distributed_ml_pytorch_amd.parallel.arena import attach_arena

    torch.manual_seed(0)
    m, _, nc = build_model(model)
    m = m.cuda()
    attach_arena(m, shadow_dtype=torch.bfloat16, channels_last=True)
    x = torch.randn(6, *shape, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    y = torch.randint(0, nc, (6,), device="cuda")
    for _ in range(3):                       # move the running stats (train mode)
        loss, _ = softmax_cross_entropy(m(x), y)
        loss.backward()
    m.eval()
    with torch.no_grad():
        ref32 = m(x.float()).float()           # fp32 ATen path, running-stats BN
        eval_fold._FOLD = False
        try:
            unfolded = m(x).float()
        finally:
            eval_fold._FOLD = True
        with eval_fold.fold_session():
            out = m(x).float()
            out2 = m(x).float()                # cached fold
    # the folded bf16 forward is as close to fp32 as the unfolded bf16 forward
    # (the two round at different points: bf16(w * s) vs the bf16 pre-BN output)
    e_fold, e_unf = _rel(out, ref32), _rel(unfolded, ref32)
    assert e_fold < 1.5 * e_unf + 5e-3, (e_fold, e_unf)
    assert _rel(out, unfolded) < 6e-2, _rel(out, unfolded)
    assert torch.equal(out, out2)
    m.train()


def test_conv_layer_autograd_and_bn_fusion():
    """Conv2d(native) -> BatchNorm2d(partials) matches the stock fp32 chain."""
    from distributed_ml_pytorch_amd.ops import layers as L

    torch.manual_seed(0)
    conv = L.Conv2d(64, 128, 3, stride=1, padding=1, bias=False).cuda()
    conv.emit_bn_stats = True
    bn = L.BatchNorm2d(128, relu=True).cuda()
    x = torch.randn(8, 64, 16, 16, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    x.requires_grad_(True)
    y = bn(conv(x))
    assert hasattr(conv(x.detach()), "_dmp_bn_part")
    xr = x.detach().float().requires_grad_(True)
    wr = conv.weight.detach().to(torch.bfloat16).float().requires_grad_(True)
    yr = F.relu(F.batch_norm(F.conv2d(xr, wr, None, 1, 1), None, None,
                             bn.weight.detach(), bn.bias.detach(), True))
    assert _rel(y, yr) < 2e-2
    g = torch.randn_like(yr)
    (y.float() * g).sum().backward()
    (yr * g).sum().backward()
    assert _rel(x.grad, xr.grad) < 3e-2
    assert _rel(conv.weight.grad, wr.grad) < 3e-2


def test_unsupported_shapes_fall_back():
    from distributed_ml_pytorch_amd.ops import layers as L

    conv = L.Conv2d(3, 64, 3, padding=1, bias=False).cuda()   # stem: CI=3 -> MIOpen
    x = torch.randn(2, 3, 8, 8, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    y = conv(x)
    yr = F.conv2d(x.float(), conv.weight.float().to(torch.bfloat16).float(), None, 1, 1)
    assert _rel(y, yr) < 1e-2


SMALL_SHAPES = [
    # B, CI, H, W, CO, k, stride, pad   (stems: CIFAR ResNet, ImageNet ResNet, AlexNet)
    (8, 3, 32, 32, 64, 3, 1, 1),
    (2, 3, 40, 36, 64, 7, 2, 3),
    (2, 3, 67, 67, 64, 11, 4, 2),
    (3, 1, 28, 28, 128, 5, 1, 2),
    (5, 3, 9, 11, 64, 3, 1, 1),        # pixel count not a multiple of 256
    (3, 3, 8, 16, 64, 3, 1, 1),        # MFMA stem (stem3_*): 384 pixels, partial blocks
    (2, 1, 16, 8, 64, 3, 1, 1),        # MFMA stem with CI = 1 (K = 9)
]


@pytest.mark.parametrize("B,CI,H,W,CO,k,st,pd", SMALL_SHAPES)
def test_small_conv_fwd_wgrad(B, CI, H, W, CO, k, st, pd):
    """Few-input-channel (stem) conv kernels vs fp32 PyTorch, both input layouts."""
    from distributed_ml_pytorch_amd.ops._ext import native

    nat = native()
    torch.manual_seed(1)
    xc = torch.randn(B, CI, H, W, device="cuda").to(torch.bfloat16)
    w = (torch.randn(CO, CI, k, k, device="cuda") / (CI * k * k) ** 0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=CL)
    wr = w.float().requires_grad_(True)
    yr = F.conv2d(xc.float(), wr, None, st, pd)
    dy = torch.randn_like(yr).to(torch.bfloat16).contiguous(memory_format=CL)
    yr.backward(dy.float())
    for x in (xc.contiguous(memory_format=CL), xc.contiguous()):
        y, part, G = nat.conv_small_fwd(x, w, st, pd, True)
        assert y.shape == yr.shape and y.is_contiguous(memory_format=CL)
        assert _rel(y, yr) < 1e-2
        ps = part[:2 * int(G) * CO].view(2, int(G), CO).sum(1)
        yf = y.float()
        torch.testing.assert_close(ps[0], yf.sum(dim=(0, 2, 3)), rtol=1e-3, atol=1e-2)
        torch.testing.assert_close(ps[1], (yf * yf).sum(dim=(0, 2, 3)), rtol=1e-3, atol=1e-2)
        dw = torch.zeros(CO, CI, k, k, device="cuda").contiguous(memory_format=CL)
        nat.conv_small_wgrad(dy, x, dw, st, pd)
        assert _rel(dw, wr.grad) < 1e-2
        nat.conv_small_wgrad(dy, x, dw, st, pd)
        assert _rel(dw, 2 * wr.grad) < 1e-2


def test_weight_transpose_batched():
    from distributed_ml_pytorch_amd.ops._ext import native

    shapes = [(64, 64, 3, 3), (128, 64, 1, 1), (512, 256, 3, 3), (64, 128, 3, 3)]
    offs, rows, off = [], [], 0
    for s in shapes:
        offs.append(off)
        rows.append([off, s[0], s[2] * s[3], s[1]])
        off += s[0] * s[1] * s[2] * s[3] + 64
    src = torch.randn(off, device="cuda").to(torch.bfloat16)
    dst = torch.zeros_like(src)
    table = torch.tensor(rows, dtype=torch.int64, device="cuda")
    native().conv_weight_transpose_batched(src, dst, table, max(s[0] * s[1] * s[2] * s[3] for s in shapes))
    for o, (co, ci, r, k) in zip(offs, shapes):
        n = co * ci * r * k
        w = src[o:o + n].view(co, r, k, ci)
        wt = dst[o:o + n].view(ci, r, k, co)
        assert torch.equal(wt, w.permute(3, 1, 2, 0))


def test_conv_layer_bias_native():
    """AlexNet-style conv with bias on the native path: output and all grads vs fp32."""
    from distributed_ml_pytorch_amd.ops import layers as L
    from distributed_ml_pytorch_amd.parallel.arena import FlatArena

    torch.manual_seed(2)
    conv = L.Conv2d(64, 192, 5, padding=2, bias=True).cuda()
    with torch.no_grad():
        conv.bias.uniform_(-0.5, 0.5)
    FlatArena(conv, device="cuda")
    x = torch.randn(4, 64, 8, 8, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    x.requires_grad_(True)
    y = conv(x)
    w = conv.weight._dmp_w16.float().detach().requires_grad_(True)
    b = conv.bias.detach().clone().requires_grad_(True)
    xr = x.detach().float().requires_grad_(True)
    yr = F.conv2d(xr, w, b, 1, 2)
    assert _rel(y, yr) < 1e-2
    dy = torch.randn_like(yr)
    y.backward(dy.to(torch.bfloat16))
    yr.backward(dy.to(torch.bfloat16).float())
    assert _rel(conv.weight.grad, w.grad) < 1e-2
    assert _rel(conv.bias.grad, b.grad) < 1e-2
    assert _rel(x.grad, xr.grad) < 1e-2


def test_subsample2_gather_and_add_back():
    """x[:, :, ::2, ::2] gather and its in-place add-back (stride-2 shortcut alias)."""
    from distributed_ml_pytorch_amd.ops._ext import native

    nat = native()
    for hw in ((15, 14), (16, 16), (1, 3)):
        x = torch.randn(3, 64, *hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        xs = nat.subsample2(x)
        assert xs.is_contiguous(memory_format=CL)
        assert torch.equal(xs, x[:, :, ::2, ::2])
        d = torch.randn_like(x.float()).to(torch.bfloat16).contiguous(memory_format=CL)
        ref = d.float().clone()
        ref[:, :, ::2, ::2] += xs.float()
        nat.add_subsampled2(d, xs)
        torch.testing.assert_close(d.float(), ref.to(torch.bfloat16).float(), rtol=0, atol=0)


@pytest.mark.parametrize("stride,cin,planes,hw", [(1, 64, 64, 16), (2, 64, 128, 16),
                                                  (2, 128, 256, 15)])
def test_resnet_block_alias_shortcut_grad(stride, cin, planes, hw):
    """BasicBlock on the native path (the shortcut's gradient is summed inside
    conv1's dgrad epilogue through the alias output; at stride 2 the 1x1
    shortcut reads conv1's subsampled alias and its gradient lands on parity
    class (0, 0), odd sizes included) vs an fp32 functional reference."""
    from distributed_ml_pytorch_amd.models.resnet import BasicBlock

    torch.manual_seed(0)
    blk = BasicBlock(cin, planes, stride).cuda()
    if stride == 2:
        _, xa = blk.conv1(torch.zeros(1, cin, hw, hw, device="cuda", dtype=torch.bfloat16)
                          .contiguous(memory_format=CL), alias="sub")
        assert xa.shape[-1] == (hw + 1) // 2, "native stride-2 conv did not subsample its alias"
    x = torch.randn(4, cin, hw, hw, device="cuda").to(torch.bfloat16)
    x = x.contiguous(memory_format=CL).requires_grad_(True)
    y = blk(x)
    g = torch.randn(y.shape, device="cuda")
    (y.float() * g).sum().backward()

    def w(conv):
        return conv.weight.detach().to(torch.bfloat16).float()

    def bn(t, m):
        return F.batch_norm(t, None, None, m.weight.detach(), m.bias.detach(), True, 0.1, m.eps)

    xr = x.detach().float().requires_grad_(True)
    h = F.relu(bn(F.conv2d(xr, w(blk.conv1), None, stride, 1), blk.bn1))
    if blk.shortcut is None:
        sc = xr
    else:
        sc = bn(F.conv2d(xr, w(blk.shortcut[0]), None, stride, 0), blk.shortcut[1])
    yr = F.relu(bn(F.conv2d(h, w(blk.conv2), None, 1, 1), blk.bn2) + sc)
    (yr * g).sum().backward()
    assert _rel(y, yr) < 3e-2
    assert _rel(x.grad, xr.grad) < 6e-2      # two bf16 conv+BN levels deep
    # the same native block with the shortcut gradient summed by autograd instead
    xb = x.detach().clone().requires_grad_(True)
    h = blk.bn1(blk.conv1(xb))
    sc = xb if blk.shortcut is None else blk.shortcut(xb)
    yb = blk.bn2(blk.conv2(h), residual=sc)
    (yb.float() * g).sum().backward()
    assert _rel(x.grad, xb.grad) < 1e-2


@pytest.mark.parametrize("stride,cin,planes", [(1, 256, 64), (2, 256, 128), (1, 64, 64)])
def test_resnet_bottleneck_block_grad(stride, cin, planes):
    """ResNet-50 Bottleneck (1x1 -> 3x3 -> 1x1, BN+ReLU fused, residual summed in
    bn3 and the shortcut gradient in conv1's dgrad) on the native path vs an fp32
    functional reference: identity shortcut, strided projection, widening
    projection."""
    from distributed_ml_pytorch_amd.models.resnet import Bottleneck

    torch.manual_seed(0)
    blk = Bottleneck(cin, planes, stride).cuda()
    x = torch.randn(4, cin, 14, 14, device="cuda").to(torch.bfloat16)
    x = x.contiguous(memory_format=CL).requires_grad_(True)
    y = blk(x)
    g = torch.randn(y.shape, device="cuda")
    (y.float() * g).sum().backward()

    def w(conv):
        return conv.weight.detach().to(torch.bfloat16).float()

    def bn(t, m):
        return F.batch_norm(t, None, None, m.weight.detach(), m.bias.detach(), True, 0.1, m.eps)

    xr = x.detach().float().requires_grad_(True)
    h = F.relu(bn(F.conv2d(xr, w(blk.conv1)), blk.bn1))
    h = F.relu(bn(F.conv2d(h, w(blk.conv2), None, stride, 1), blk.bn2))
    sc = xr if blk.shortcut is None else bn(F.conv2d(xr, w(blk.shortcut[0]), None, stride),
                                            blk.shortcut[1])
    yr = F.relu(bn(F.conv2d(h, w(blk.conv3)), blk.bn3) + sc)
    (yr * g).sum().backward()
    assert _rel(y, yr) < 3e-2
    assert _rel(x.grad, xr.grad) < 8e-2      # three bf16 conv+BN levels deep
    for conv in (blk.conv1, blk.conv2, blk.conv3):
        assert torch.isfinite(conv.weight.grad).all()
    # weight gradient of the last conv (one level deep) against the oracle
    wr3 = w(blk.conv3).requires_grad_(True)
    h2 = h.detach()
    yr3 = F.relu(bn(F.conv2d(h2, wr3), blk.bn3) + sc.detach())
    (yr3 * g).sum().backward()
    assert _rel(blk.conv3.weight.grad, wr3.grad) < 6e-2


def test_conv1x1_gemm_route(monkeypatch):
    """1x1 / stride-1 convs routed to the MFMA GEMM (ops/conv.py _GEMM_ROUTE):
    forward + BN partial sums from the GEMM store epilogue, data gradient (+ the
    shortcut-alias addend), weight gradient accumulated in fp32 -- helpers and
    the full layer with the route forced, vs fp32."""
    from distributed_ml_pytorch_amd.ops import conv as C
    from distributed_ml_pytorch_amd.ops import layers as L

    torch.manual_seed(0)
    B, CI, H, W, CO = 8, 256, 14, 14, 64
    x = torch.randn(B, CI, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(CO, CI, 1, 1, device="cuda") / CI ** 0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=CL)
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    yr = F.conv2d(xr, wr)
    dy = torch.randn_like(yr).to(torch.bfloat16).contiguous(memory_format=CL)
    yr.backward(dy.float())
    part = torch.zeros(2 * C.BN_SLOTS * CO + C.BN_TAIL, device="cuda")
    y = C._gemm1x1_fwd(x, w, part)
    assert y.is_contiguous(memory_format=CL)
    assert _rel(y, yr) < 1e-2
    ps = part[:2 * C.BN_SLOTS * CO].view(2, C.BN_SLOTS, CO).sum(1)
    yf = y.float()
    torch.testing.assert_close(ps[0], yf.sum(dim=(0, 2, 3)), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(ps[1], (yf * yf).sum(dim=(0, 2, 3)), rtol=1e-3, atol=1e-2)
    dx = C._gemm1x1_dgrad(dy, w)
    assert _rel(dx, xr.grad) < 1e-2
    add = torch.randn_like(x)
    assert _rel(C._gemm1x1_dgrad(dy, w, add), xr.grad + add.float()) < 1e-2
    g = torch.zeros(CO, CI, 1, 1, device="cuda").contiguous(memory_format=CL)
    C._gemm1x1_wgrad(dy, x, g)
    assert _rel(g, wr.grad) < 1e-2
    # the whole layer with every pass forced onto the GEMM route
    monkeypatch.setattr(C, "_fwd_cfg", lambda *a: C._GEMM_ROUTE)
    monkeypatch.setattr(C, "_dgrad_cfg", lambda *a: C._GEMM_ROUTE)
    monkeypatch.setattr(C, "_wgrad_cfg", lambda *a: C._GEMM_ROUTE)
    conv = L.Conv2d(CI, CO, 1, bias=False).cuda()
    with torch.no_grad():
        conv.weight.copy_(w.float())
    xa = x.detach().clone().requires_grad_(True)
    yl = conv(xa)
    yl.backward(dy)
    assert _rel(yl, yr) < 1e-2
    assert _rel(xa.grad, xr.grad) < 1e-2
    assert _rel(conv.weight.grad, wr.grad) < 1e-2


@pytest.mark.parametrize("B,CI,H,CO,st", [(8, 256, 8, 256, 1), (4, 128, 16, 256, 2),
                                          (6, 64, 5, 128, 1)])
def test_conv_im2col_wgrad_route(monkeypatch, B, CI, H, CO, st):
    """3x3 weight gradient as patch matrix x wgrad GEMM (ops/conv.py _IM2COL_ROUTE):
    the helper accumulating into a channels_last fp32 gradient, and a whole layer
    with the route forced, vs fp32."""
    from distributed_ml_pytorch_amd.ops import conv as C
    from distributed_ml_pytorch_amd.ops import layers as L

    monkeypatch.setattr(C, "_IM2COL_WGRAD", True)     # opt-in route
    torch.manual_seed(3)
    x = torch.randn(B, CI, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(CO, CI, 3, 3, device="cuda") / (9 * CI) ** 0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=CL)
    wr = w.float().requires_grad_(True)
    yr = F.conv2d(x.float(), wr, None, st, 1)
    dy = torch.randn_like(yr).to(torch.bfloat16).contiguous(memory_format=CL)
    yr.backward(dy.float())
    assert C._im2col_wgrad_ok(x, tuple(w.shape), st, 1)
    g = torch.zeros(CO, CI, 3, 3, device="cuda").contiguous(memory_format=CL)
    C._im2col_wgrad(dy, x, g, st, 1)
    assert _rel(g, wr.grad) < 1e-2
    C._im2col_wgrad(dy, x, g, st, 1)                 # accumulates
    assert _rel(g, 2 * wr.grad) < 1e-2
    monkeypatch.setattr(C, "_wgrad_cfg", lambda *a: C._IM2COL_ROUTE)
    conv = L.Conv2d(CI, CO, 3, stride=st, padding=1, bias=False).cuda()
    with torch.no_grad():
        conv.weight.copy_(w.float())
    conv(x.detach().clone().requires_grad_(True)).backward(dy)
    assert _rel(conv.weight.grad, wr.grad) < 1e-2


@pytest.mark.parametrize("B,H", [(2, 224), (3, 48), (1, 8)])
def test_stem_conv_fwd_stats_wgrad(B, H):
    """ImageNet 7x7/2/3 stem (space-to-depth MFMA kernels) vs fp32 PyTorch."""
    from distributed_ml_pytorch_amd.ops._ext import native

    nat = native()
    W = 224
    assert nat.stem_supported(H, W) and not nat.stem_supported(H + 2, W)
    assert not nat.stem_supported(H, 232)
    torch.manual_seed(2)
    x = torch.randn(B, 3, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(64, 3, 7, 7, device="cuda") / 147 ** 0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=CL)
    wr = w.float().requires_grad_(True)
    yr = F.conv2d(x.float(), wr, None, 2, 3)
    dy = torch.randn_like(yr).to(torch.bfloat16).contiguous(memory_format=CL)
    yr.backward(dy.float())
    y, part, xs = nat.stem_fwd(x, w, True)
    assert y.shape == yr.shape and y.is_contiguous(memory_format=CL)
    assert _rel(y, yr) < 1e-2
    ps = part[:2 * 64 * 64].view(2, 64, 64).sum(1)
    yf = y.float()
    torch.testing.assert_close(ps[0], yf.sum(dim=(0, 2, 3)), rtol=2e-3, atol=5e-2)
    torch.testing.assert_close(ps[1], (yf * yf).sum(dim=(0, 2, 3)), rtol=2e-3, atol=5e-2)
    y2, none, _ = nat.stem_fwd(x, w, False)
    assert none is None or none.numel() == 0
    assert torch.equal(y2, y)
    dw = torch.zeros(64, 3, 7, 7, device="cuda").contiguous(memory_format=CL)
    nat.stem_wgrad(dy, xs, dw)
    assert _rel(dw, wr.grad) < 1e-2
    nat.stem_wgrad(dy, xs, dw)
    assert _rel(dw, 2 * wr.grad) < 1e-2


def test_stem_conv_layer_route():
    """ops.conv2d routes the ResNet stem to the native stem kernels (arena-less
    master: the weight gradient comes back through autograd)."""
    from distributed_ml_pytorch_amd.ops import conv as C

    torch.manual_seed(3)
    x = torch.randn(2, 3, 64, 224, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    master = torch.nn.Parameter((torch.randn(64, 3, 7, 7, device="cuda") / 147 ** 0.5)
                                .contiguous(memory_format=CL))
    assert C.stem_conv_supported(x, master, 2, 3, 1, 1)
    slots = torch.zeros(2 * 64 * 64 + 4, device="cuda")
    y = C.conv2d(x, None, None, 2, 3, 1, 1, master=master, want_stats=True, slots=slots)
    assert hasattr(y, "_dmp_bn_part")
    dy = torch.randn_like(y.float())
    y.float().backward(dy)
    wr = master.detach().to(torch.bfloat16).float().requires_grad_(True)
    yr = F.conv2d(x.float(), wr, None, 2, 3)
    yr.backward(dy.to(torch.bfloat16).float())
    assert _rel(y, yr) < 1e-2
    assert _rel(master.grad, wr.grad) < 1e-2


def _grads_with_bn_fusion(monkeypatch, fuse, model, x, g, bitmask=True):
    from distributed_ml_pytorch_amd.ops import functional as Fn

    monkeypatch.setattr(Fn, "_BN_BWD_FUSE", fuse if fuse else "0")
    monkeypatch.setattr(Fn, "_BN_BITMASK", bitmask)
    for p in model.parameters():
        p.grad = None
    xx = x.detach().clone().requires_grad_(True)
    y = model(xx)
    (y.float() * g).sum().backward()
    torch.cuda.synchronize()
    return y.detach(), [xx.grad] + [p.grad.detach().clone() for p in model.parameters()]


@pytest.mark.parametrize("kind", ["basic_s1", "basic_s2", "bottleneck"])
def test_bn_backward_fused_into_dgrad(kind, monkeypatch):
    """BN(+ReLU) backward reductions run in the consuming conv's dgrad epilogue
    (csrc/conv.hip bnb_*; ops/functional.py BNLink): gradients match the
    separate reduce pass.  Two chained blocks exercise both ReLU-mask sources:
    bn1 -> conv2 (mask recomputed from x) and block 1's bn2 + residual ->
    block 2's conv1 with the shortcut gradient as the dgrad addend (mask from
    the stored output)."""
    from distributed_ml_pytorch_amd.models.resnet import BasicBlock, Bottleneck
    from distributed_ml_pytorch_amd.ops import functional as Fn

    torch.manual_seed(0)
    if kind == "bottleneck":
        model = torch.nn.Sequential(Bottleneck(256, 64, 1), Bottleneck(256, 128, 2)).cuda()
        x = torch.randn(4, 256, 14, 14, device="cuda")
    else:
        s = 1 if kind == "basic_s1" else 2
        model = torch.nn.Sequential(BasicBlock(64, 64, 1), BasicBlock(64, 64 * s, s)).cuda()
        x = torch.randn(4, 64, 16, 16, device="cuda")
    x = x.to(torch.bfloat16).contiguous(memory_format=CL)
    g = torch.randn(model(x).shape, device="cuda")
    # reference: standalone reduce, ReLU mask of the residual BNs read from y
    y0, ref = _grads_with_bn_fusion(monkeypatch, False, model, x, g, bitmask=False)
    # standalone reduce with the forward's 1-bit mask
    _, bits = _grads_with_bn_fusion(monkeypatch, False, model, x, g)
    for a, b in zip(ref, bits):
        assert _rel(b, a) < 5e-3
    before = dict(Fn.BN_BWD_FUSE_STATS)
    y1, got = _grads_with_bn_fusion(monkeypatch, "all", model, x, g)
    assert Fn.BN_BWD_FUSE_STATS["fused"] > before["fused"]
    assert _rel(y1, y0) < 1e-3        # forward untouched (atomic-order noise only)
    for a, b in zip(ref, got):
        assert _rel(b, a) < 5e-3
    # the default policy (residual BNs only)
    _, res = _grads_with_bn_fusion(monkeypatch, "residual", model, x, g)
    for a, b in zip(ref, res):
        assert _rel(b, a) < 5e-3
    # a second identical step: persistent slot buffers were left zeroed
    _, again = _grads_with_bn_fusion(monkeypatch, "all", model, x, g)
    for a, b in zip(got, again):
        assert _rel(b, a) < 5e-3


def test_bn_backward_fusion_falls_back_on_shared_output(monkeypatch):
    """A BN output read by two convs: each conv's dgrad records a fused
    reduction, autograd sums the two input gradients, and the BN backward must
    notice (different tensor) and redo the reduce over the summed gradient."""
    from distributed_ml_pytorch_amd.ops import functional as Fn
    from distributed_ml_pytorch_amd.ops.layers import BatchNorm2d, Conv2d

    class Fork(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.conv0 = Conv2d(64, 64, 3, 1, 1, bias=False)
            self.bn = BatchNorm2d(64, relu=True)
            self.a = Conv2d(64, 64, 3, 1, 1, bias=False)
            self.b = Conv2d(64, 64, 1, 1, 0, bias=False)

        def forward(self, x):
            h = self.bn(self.conv0(x))
            return self.a(h) + self.b(h)

    torch.manual_seed(0)
    model = Fork().cuda()
    x = torch.randn(4, 64, 16, 16, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    g = torch.randn(4, 64, 16, 16, device="cuda")
    _, ref = _grads_with_bn_fusion(monkeypatch, False, model, x, g)
    before = dict(Fn.BN_BWD_FUSE_STATS)
    _, got = _grads_with_bn_fusion(monkeypatch, "all", model, x, g)
    assert Fn.BN_BWD_FUSE_STATS["fallback"] > before["fallback"]
    for a, b in zip(ref, got):
        assert _rel(b, a) < 5e-3


@pytest.mark.parametrize("B,CI,H,CO", [(4, 64, 32, 128), (2, 128, 16, 256), (8, 256, 8, 512),
                                       (2, 64, 56, 128)])
def test_stride2_halo_dgrad_configs(B, CI, H, CO):
    """3x3/stride-2 data gradient as parity-class halo tiles (conv_dgrad_s2_kernel):
    every applicable config vs fp32, plain, with a full-resolution addend, and with
    the subsampled shortcut addend (class (0, 0) only)."""
    from distributed_ml_pytorch_amd.ops._ext import native

    nat = native()
    torch.manual_seed(0)
    OH = H // 2
    w = (torch.randn(CO, CI, 3, 3, device="cuda") / (CI * 9) ** 0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=CL)
    dy = torch.randn(B, CO, OH, OH, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    ref = torch.nn.grad.conv2d_input((B, CI, H, H), w.float(), dy.float(), stride=2, padding=1)
    add = torch.randn(B, CI, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    sub = torch.randn(B, CI, OH, OH, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    ref_sub = ref.clone()
    ref_sub[:, :, ::2, ::2] += sub.float()
    cfgs = list(nat.conv_dgrad_s2_configs(H, H, OH, OH, CO, CI, 3, 3, 2, 1))
    assert cfgs, "no stride-2 halo config applies"
    for cfg in cfgs:
        dx = nat.conv_dgrad(dy, w, H, H, 2, 1, cfg)
        assert _rel(dx, ref) < 1e-2, cfg
        dxa = nat.conv_dgrad(dy, w, H, H, 2, 1, cfg, None, add)
        assert _rel(dxa, ref + add.float()) < 1e-2, cfg
        dxs = nat.conv_dgrad(dy, w, H, H, 2, 1, cfg, addend=sub, addend_sub=True)
        assert _rel(dxs, ref_sub) < 1e-2, cfg


@pytest.mark.parametrize("B,C,H", [(4, 64, 32), (3, 128, 16), (8, 256, 8), (8, 512, 4)])
def test_dgrad_addend_bitmask(B, C, H):
    """Deferred residual mask (ops/functional.py): the data-gradient epilogue
    applying the 1-bit ReLU mask to its addend (ConvArgs::addmask) == the same
    dgrad with the addend masked beforehand, bitwise, on every tile family that
    takes an addend: halo tiles (row-staged epilogue), the persistent 64-channel
    kernel (hand-counted mask loads) and the implicit GEMM."""
    from distributed_ml_pytorch_amd.ops._ext import native
    from distributed_ml_pytorch_amd.ops.functional import apply_bitmask

    nat = native()
    torch.manual_seed(3)
    dy = torch.randn(B, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(C, C, 3, 3, device="cuda") / (C * 9) ** 0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=CL)
    add = torch.randn_like(dy)
    mask = torch.randint(0, 256, (B * H * H * C // 8,), device="cuda", dtype=torch.uint8)
    masked = apply_bitmask(add, mask).contiguous(memory_format=CL)
    # the torch fallback itself against an explicit bit unpack
    bits = torch.stack([(mask >> k) & 1 for k in range(8)], 1).view(B, H, H, C).permute(0, 3, 1, 2)
    assert torch.equal(masked.float(), torch.where(bits.bool(), add.float(), 0.0))
    cfgs = list(nat.conv_halo_configs(H, H, C, 3, 3, 1, 1)) + [0, 3, -1]
    for cfg in cfgs:
        ref = nat.conv_dgrad(dy, w, H, H, 1, 1, cfg, None, masked)
        got = nat.conv_dgrad(dy, w, H, H, 1, 1, cfg, None, add, addend_mask=mask)
        assert torch.equal(got, ref), (cfg, (got.float() - ref.float()).abs().max())


@pytest.mark.parametrize("stride,cin,planes", [(1, 64, 64), (2, 64, 128)])
def test_resnet_block_deferred_dres(stride, cin, planes, monkeypatch):
    """BasicBlock backward with bn2's residual gradient handed over unmasked
    (identity: into conv1's dgrad epilogue; projection: into the shortcut BN's
    mode-3 passes) == the materialised-dres path (DMP_BN_DEFER_RES=0), and
    nothing is materialised on the way."""
    from distributed_ml_pytorch_amd.models.resnet import BasicBlock
    from distributed_ml_pytorch_amd.ops import functional as Fn

    torch.manual_seed(0)
    blk = BasicBlock(cin, planes, stride).cuda()
    x0 = torch.randn(8, cin, 16, 16, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    g = torch.randn(8, planes, 16 // stride, 16 // stride, device="cuda")
    grads = {}
    for defer in (False, True):
        monkeypatch.setattr(Fn, "_BN_DEFER_RES", defer)
        before = dict(Fn.DEFER_RES_STATS)
        blk.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        (blk(x).float() * g).sum().backward()
        torch.cuda.synchronize()
        grads[defer] = [x.grad.float()] + [p.grad.float() for p in blk.parameters()]
        d = {k: Fn.DEFER_RES_STATS[k] - before[k] for k in before}
        if defer:
            assert d["deferred"] == 1 and d["native"] == 1 and d["materialized"] == 0, d
        else:
            assert d["deferred"] == 0, d
    for a, b in zip(grads[False], grads[True]):
        # fp32 atomics order the BN / wgrad sums differently run to run
        assert _rel(b, a) < 5e-3, _rel(b, a)


@pytest.mark.parametrize("stride,cin,planes", [(1, 256, 64), (2, 256, 128)])
def test_bottleneck_deferred_dres(stride, cin, planes, monkeypatch):
    """Bottleneck backward with bn3's residual gradient deferred: identity shortcut ->
    conv1's 1x1 data gradient (GEMM route or implicit GEMM) masks its addend in the
    epilogue; projection -> the shortcut BN's mode-3 passes.  Matches the
    materialised-dres path, nothing materialised."""
    from distributed_ml_pytorch_amd.models.resnet import Bottleneck
    from distributed_ml_pytorch_amd.ops import functional as Fn

    torch.manual_seed(0)
    blk = Bottleneck(cin, planes, stride).cuda()
    x0 = torch.randn(4, cin, 14, 14, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    oh = (14 + stride - 1) // stride
    g = torch.randn(4, planes * 4, oh, oh, device="cuda")
    grads = {}
    for defer in (False, True):
        monkeypatch.setattr(Fn, "_BN_DEFER_RES", defer)
        before = dict(Fn.DEFER_RES_STATS)
        blk.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        (blk(x).float() * g).sum().backward()
        torch.cuda.synchronize()
        grads[defer] = [x.grad.float()] + [p.grad.float() for p in blk.parameters()]
        d = {k: Fn.DEFER_RES_STATS[k] - before[k] for k in before}
        if defer:
            assert d["deferred"] == 1 and d["native"] == 1 and d["materialized"] == 0, d
        else:
            assert d["deferred"] == 0, d
    for a, b in zip(grads[False], grads[True]):
        assert _rel(b, a) < 5e-3, _rel(b, a)


@pytest.mark.parametrize("kind", ["basic32", "bottleneck256"])
def test_residual_mark_on_bn_output_input(kind, monkeypatch):
    """a block whose input is a native BatchNorm output.  For
    BasicBlock(32, 32) conv1 is off the native path and hands x itself back as the
    shortcut, which also feeds conv1: the residual must NOT be marked single-use
    (bn2 would hand its unmasked dY over tagged, autograd would sum it with conv1's
    dx and drop the mask).  Gradients with the deferred mask == DMP_BN_DEFER_RES=0."""
    from distributed_ml_pytorch_amd.models.resnet import BasicBlock, Bottleneck
    from distributed_ml_pytorch_amd.ops import functional as Fn
    from distributed_ml_pytorch_amd.ops import layers as L

    torch.manual_seed(0)
    if kind == "basic32":
        C, blk, hw = 32, BasicBlock(32, 32, 1), 16
    else:
        C, blk, hw = 256, Bottleneck(256, 64, 1), 14
    pre = L.BatchNorm2d(C, relu=True).cuda()
    blk = blk.cuda()
    x0 = torch.randn(4, C, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    g = torch.randn(4, C, hw, hw, device="cuda")
    grads = {}
    for defer in (False, True):
        monkeypatch.setattr(Fn, "_BN_DEFER_RES", defer)
        blk.zero_grad(set_to_none=True)
        pre.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        (blk(pre(x)).float() * g).sum().backward()
        torch.cuda.synchronize()
        grads[defer] = [x.grad.float()] + [p.grad.float() for p in
                                           list(pre.parameters()) + list(blk.parameters())]
    for a, b in zip(grads[False], grads[True]):
        assert _rel(b, a) < 5e-3, _rel(b, a)
