"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CL = torch.channels_last


@pytest.fixture(scope="module")
def nat():
    from distributed_ml_pytorch_amd.ops._ext import native

    return native()


def _bf(x):
    return x.to(torch.bfloat16)


# ------------------------------------------------------------------- optimizer
@pytest.mark.parametrize("momentum,wd,nesterov", [(0.0, 0.0, False), (0.9, 5e-4, False),
                                                  (0.9, 0.0, True)])
def test_asgd_fused_step(nat, momentum, wd, nesterov):
    n = 4096 * 7 + 64
    g = torch.randn(n, device="cuda")
    p = torch.randn(n, device="cuda")
    acc = torch.randn(n, device="cuda")
    mom = torch.randn(n, device="cuda") if momentum else None
    w16 = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    lr = 0.1
    # reference
    d = g + wd * p
    rm = None
    if momentum:
        rm = momentum * mom + d
        d = d + momentum * rm if nesterov else rm
    rp = p - lr * d
    racc = acc - lr * d
    nat.asgd_fused_step(g, p, acc, mom, w16, lr, wd, momentum, 0.0, nesterov)
    torch.testing.assert_close(p, rp, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(acc, racc, rtol=1e-6, atol=1e-6)
    if momentum:
        torch.testing.assert_close(mom, rm, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(w16, p.to(torch.bfloat16), rtol=0, atol=0)


def test_ps_apply_atomic_concurrent_streams(nat):
    """fp32-atomic PS apply (completion-ordered central / sharded PS): four
    deltas applied at once from four streams all land (fp32 reference, order
    free, so a tolerance); fp32 and bf16 wire deltas."""
    n = (1 << 20) + 4
    shard = torch.randn(n, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(1)
    deltas = [torch.randn(n, device="cuda", generator=g) for _ in range(3)]
    deltas.append(torch.randn(n, device="cuda", generator=g).to(torch.bfloat16))
    ref = shard.double() + sum(0.25 * d.double() for d in deltas)
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in deltas]
    for s, d in zip(streams, deltas):
        with torch.cuda.stream(s):
            nat.ps_apply(shard, d, None, 0.25, True)
    torch.cuda.synchronize()
    torch.testing.assert_close(shard.double(), ref, rtol=1e-5, atol=1e-5)
    with pytest.raises(RuntimeError):
        nat.ps_apply(shard, deltas[0], torch.empty(n, device="cuda", dtype=torch.bfloat16),
                     1.0, True)


def test_ps_apply_and_pull_land(nat):
    n = 1 << 16
    shard = torch.randn(n, device="cuda")
    delta = torch.randn(n, device="cuda")
    ref = shard + 0.5 * delta
    mirror = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    nat.ps_apply(shard, delta, mirror, 0.5)
    torch.testing.assert_close(shard, ref)
    torch.testing.assert_close(mirror, ref.to(torch.bfloat16), rtol=0, atol=0)
    d16 = delta.to(torch.bfloat16)
    ref2 = shard + d16.float()
    nat.ps_apply(shard, d16, None, 1.0)
    torch.testing.assert_close(shard, ref2)
    p = torch.empty(n, device="cuda")
    acc = torch.randn(n, device="cuda")
    w16 = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    nat.pull_land(p, shard, acc, w16)
    torch.testing.assert_close(p, shard + acc)
    nat.pull_land(p, shard, None, w16)
    torch.testing.assert_close(p, shard)
    torch.testing.assert_close(w16, shard.to(torch.bfloat16), rtol=0, atol=0)


def test_push_handoff_and_sumsq(nat):
    n = 1 << 15
    acc = torch.randn(n, device="cuda")
    ref = acc.clone()
    o32 = torch.empty_like(acc)
    o16 = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    nat.push_handoff(acc, o32, o16)
    torch.testing.assert_close(o32, ref)
    torch.testing.assert_close(o16, ref.to(torch.bfloat16), rtol=0, atol=0)
    assert int((acc != 0).sum()) == 0
    x = torch.randn(n, device="cuda")
    torch.testing.assert_close(nat.sumsq(x), (x.double() ** 2).sum().float(), rtol=1e-4, atol=1e-3)


def test_native_rejects_bad_shapes(nat):
    with pytest.raises(RuntimeError):
        nat.asgd_fused_step(torch.zeros(6, device="cuda"), torch.zeros(6, device="cuda"),
                            None, None, None, 0.1, 0.0, 0.0, 0.0, False)
    with pytest.raises(RuntimeError):
        nat.bn_fwd(torch.zeros(2, 12, 4, 4, device="cuda", dtype=torch.bfloat16)
                   .contiguous(memory_format=CL), None, None, None, None, None, 0.1, 1e-5,
                   True, False)


# --------------------------------------------------------------- cross entropy
@pytest.mark.parametrize("B,C,dtype,ls", [(64, 10, torch.bfloat16, 0.0), (256, 10, torch.float32, 0.0),
                                          (1000, 1000, torch.bfloat16, 0.0), (3, 130, torch.float32, 0.0),
                                          (2500, 10, torch.bfloat16, 0.0), (512, 32, torch.float32, 0.1),
                                          (300, 33, torch.float32, 0.1), (77, 1, torch.float32, 0.0),
                                          (128, 1000, torch.bfloat16, 0.1), (8, 1000, torch.float32, 0.0),
                                          (40, 2000, torch.bfloat16, 0.0), (10, 1500, torch.float32, 0.0)])
def test_softmax_xent(B, C, dtype, ls):
    from distributed_ml_pytorch_amd.ops.functional import softmax_cross_entropy

    logits = (torch.randn(B, C, device="cuda") * 3).to(dtype).requires_grad_(True)
    y = torch.randint(0, C, (B,), device="cuda")
    loss, hits = softmax_cross_entropy(logits, y, ls)
    loss.backward()
    ref_in = logits.detach().float().requires_grad_(True)
    ref = F.cross_entropy(ref_in, y, label_smoothing=ls)
    ref.backward()
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    torch.testing.assert_close(loss.float(), ref, rtol=tol, atol=tol)
    torch.testing.assert_close(logits.grad.float(), ref_in.grad, rtol=tol, atol=tol / 10)
    assert int(hits) == int((ref_in.argmax(1) == y).sum())


# ------------------------------------------------------------------ batchnorm
@pytest.mark.parametrize("shape,relu,res", [((8, 64, 16, 16), True, False),
                                            ((4, 128, 8, 8), True, True),
                                            ((16, 512, 4, 4), False, True),
                                            ((2, 192, 5, 7), False, False)])
def test_bn_act_fwd_bwd(shape, relu, res):
    from distributed_ml_pytorch_amd.ops.functional import batch_norm_act

    C = shape[1]
    x = torch.randn(shape, device="cuda") * 2 + 0.5
    r = torch.randn(shape, device="cuda") if res else None
    gamma = (torch.rand(C, device="cuda") + 0.5).requires_grad_(True)
    beta = torch.randn(C, device="cuda").requires_grad_(True)
    rm = torch.zeros(C, device="cuda")
    rv = torch.ones(C, device="cuda")
    xb = _bf(x).contiguous(memory_format=CL).requires_grad_(True)
    rb = _bf(r).contiguous(memory_format=CL).requires_grad_(True) if res else None
    y = batch_norm_act(xb, gamma, beta, rm, rv, True, 0.1, 1e-5, relu=relu, residual=rb)
    # fp32 reference on the SAME bf16-rounded inputs
    xr = xb.detach().float().requires_grad_(True)
    rr = rb.detach().float().requires_grad_(True) if res else None
    g2 = gamma.detach().clone().requires_grad_(True)
    b2 = beta.detach().clone().requires_grad_(True)
    rm2 = torch.zeros(C, device="cuda")
    rv2 = torch.ones(C, device="cuda")
    yr = F.batch_norm(xr, rm2, rv2, g2, b2, True, 0.1, 1e-5)
    if res:
        yr = yr + rr
    if relu:
        yr = F.relu(yr)
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(rm, rm2, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(rv, rv2, rtol=1e-4, atol=1e-4)
    dy = torch.randn(shape, device="cuda")
    (y.float() * dy).sum().backward()
    (yr * dy).sum().backward()
    torch.testing.assert_close(xb.grad.float(), xr.grad, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(gamma.grad, g2.grad, rtol=2e-2, atol=2e-1)
    torch.testing.assert_close(beta.grad, b2.grad, rtol=2e-2, atol=2e-1)
    if res:
        torch.testing.assert_close(rb.grad.float(), rr.grad, rtol=2e-2, atol=2e-2)


def _bn_ref(xb, mod, rb=None, relu=True):
    xr = xb.detach().float().requires_grad_(True)
    g2 = mod.weight.detach().clone().requires_grad_(True)
    b2 = mod.bias.detach().clone().requires_grad_(True)
    yr = F.batch_norm(xr, None, None, g2, b2, True, 0.1, mod.eps)
    if rb is not None:
        yr = yr + rb.detach().float()
    return (F.relu(yr) if relu else yr), xr, g2, b2


@pytest.mark.parametrize("C,res", [(64, False), (128, True), (24, False), (80, True), (96, False)])
def test_bn_fold_persistent_slots_multi_step(C, res):
    """Finalize folded into the apply passes with the layer's persistent slot
    buffers: the forward apply zeroes the backward slots and vice versa, so
    several steps in a row -- with a forward-only (no backward) pass in between --
    must each match an fp32 reference (stale sums would shift the statistics)."""
    from distributed_ml_pytorch_amd.ops import functional as DF
    from distributed_ml_pytorch_amd.ops import layers as L

    assert DF._BN_FOLD, "fold path is the default"
    torch.manual_seed(C)
    bn = L.BatchNorm2d(C, relu=True).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.normal_()
    for it in range(4):
        x = _bf(torch.randn(6, C, 9, 7, device="cuda") * (1 + it) + it).contiguous(
            memory_format=CL).requires_grad_(True)
        rb = _bf(torch.randn(6, C, 9, 7, device="cuda")).contiguous(memory_format=CL) if res else None
        bn.weight.grad = None
        bn.bias.grad = None
        y = bn(x, residual=rb)
        yr, xr, g2, b2 = _bn_ref(x, bn, rb)
        torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
        if it == 1:
            continue            # forward only: its slot sums stay behind (dirty)
        dy = torch.randn_like(yr)
        (y.float() * dy).sum().backward()
        (yr * dy).sum().backward()
        torch.testing.assert_close(x.grad.float(), xr.grad, rtol=3e-2, atol=3e-2)
        torch.testing.assert_close(bn.weight.grad, g2.grad, rtol=2e-2, atol=2e-1)
        torch.testing.assert_close(bn.bias.grad, b2.grad, rtol=2e-2, atol=2e-1)


def test_bn_fold_with_conv_producer_multi_step():
    """Conv epilogue BN partials -> folded BN apply, three steps with a
    forward-only pass in between (the conv's slot buffer is re-zeroed)."""
    from distributed_ml_pytorch_amd.ops import layers as L

    torch.manual_seed(3)
    conv = L.Conv2d(64, 64, 3, padding=1, bias=False).cuda()
    conv.emit_bn_stats = True
    bn = L.BatchNorm2d(64, relu=True).cuda()
    w16 = conv.weight.detach().to(torch.bfloat16).float()
    for it in range(4):
        x = _bf(torch.randn(8, 64, 12, 12, device="cuda")).contiguous(memory_format=CL)
        h = conv(x)
        assert getattr(h, "_dmp_bn_part", None) is not None, "conv did not emit BN partials"
        y = bn(h)
        hr = F.conv2d(x.float(), w16, padding=1)
        yr = F.relu(F.batch_norm(hr, None, None, bn.weight.detach(), bn.bias.detach(), True))
        torch.testing.assert_close(y.float(), yr, rtol=3e-2, atol=3e-2)
        if it != 1:
            y.float().sum().backward()


def test_bn_eval_uses_running_stats():
    from distributed_ml_pytorch_amd.ops.functional import batch_norm_act

    C = 64
    x = _bf(torch.randn(4, C, 8, 8, device="cuda")).contiguous(memory_format=CL)
    gamma = torch.rand(C, device="cuda") + 0.5
    beta = torch.randn(C, device="cuda")
    rm = torch.randn(C, device="cuda")
    rv = torch.rand(C, device="cuda") + 0.5
    y = batch_norm_act(x, gamma, beta, rm, rv, False, 0.1, 1e-5, relu=True)
    yr = F.relu(F.batch_norm(x.float(), rm, rv, gamma, beta, False, 0.1, 1e-5))
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)


# -------------------------------------------------------------------- pooling
def test_global_avg_pool():
    from distributed_ml_pytorch_amd.ops.functional import global_avg_pool

    x = _bf(torch.randn(32, 512, 4, 4, device="cuda")).contiguous(memory_format=CL)
    x.requires_grad_(True)
    y = global_avg_pool(x)
    xr = x.detach().float().requires_grad_(True)
    yr = xr.mean(dim=(2, 3))
    torch.testing.assert_close(y.float(), yr, rtol=1e-2, atol=1e-2)
    dy = torch.randn_like(yr)
    (y.float() * dy).sum().backward()
    (yr * dy).sum().backward()
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=1e-2, atol=1e-3)


@pytest.mark.parametrize("shape,k,st,pd", [((8, 64, 8, 8), 2, 2, 0), ((4, 192, 5, 5), 2, 2, 0),
                                           ((2, 16, 9, 9), 3, 3, 0), ((2, 64, 16, 16), 3, 2, 1),
                                           ((3, 64, 15, 15), 3, 2, 1), ((2, 8, 11, 7), 5, 2, 2)])
def test_max_pool(shape, k, st, pd):
    from distributed_ml_pytorch_amd.ops.functional import max_pool2d

    x = _bf(torch.randn(shape, device="cuda")).contiguous(memory_format=CL).requires_grad_(True)
    y = max_pool2d(x, k, st, pd)
    xr = x.detach().float().requires_grad_(True)
    yr = F.max_pool2d(xr, k, st, pd)
    torch.testing.assert_close(y.float(), yr, rtol=0, atol=0)
    dy = _bf(torch.randn_like(yr)).float()      # the native backward sees bf16 dy
    (y.float() * dy).sum().backward()
    (yr * dy).sum().backward()
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("shape", [(4, 64, 16, 16), (2, 64, 15, 17), (3, 128, 12, 9),
                                   (2, 64, 112, 112)])
def test_bn_relu_maxpool_fused(shape, monkeypatch):
    """Fused BN + ReLU + max pool 3x3/s2/p1 (csrc/bn.hip, the ImageNet stem):
    pooled output bit-identical to the unfused BN apply + max pool, gradients and
    running statistics against both the unfused kernels and fp32 PyTorch; the
    backward reduce against its exact value from the saved winning-tap x."""
    from distributed_ml_pytorch_amd.ops import functional as DF
    from distributed_ml_pytorch_amd.ops import layers as L

    torch.manual_seed(1)
    C = shape[1]
    x0 = _bf(torch.randn(shape, device="cuda") * 2 + 0.3).contiguous(memory_format=CL)
    dp = _bf(torch.randn(shape[0], C, (shape[2] - 1) // 2 + 1, (shape[3] - 1) // 2 + 1,
                         device="cuda")).float()

    gw = torch.rand(C) + 0.5
    gw[::7] *= -1                                  # negative scales: max != scale * max
    gb = torch.randn(C) * 0.2

    def make():
        bn = L.BatchNorm2d(C, relu=True).cuda()
        with torch.no_grad():
            bn.weight.copy_(gw)
            bn.bias.copy_(gb)
        return bn

    bn_f, bn_u = make(), make()
    assert DF.bn_relu_maxpool_ok(x0, bn_f, 3, 2, 1)
    xf = x0.clone().requires_grad_(True)
    yf = DF.bn_relu_maxpool(xf, bn_f, 3, 2, 1)
    (yf.float() * dp).sum().backward()

    monkeypatch.setattr(DF, "_BN_POOL_FUSE", False)
    assert not DF.bn_relu_maxpool_ok(x0, bn_u, 3, 2, 1)
    xu = x0.clone().requires_grad_(True)
    yu = DF.max_pool2d(bn_u(xu), 3, 2, 1)
    (yu.float() * dp).sum().backward()

    assert yf.shape == yu.shape and yf.is_contiguous(memory_format=CL)
    assert torch.equal(yf, yu)
    torch.testing.assert_close(bn_f.running_mean, bn_u.running_mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(bn_f.running_var, bn_u.running_var, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(xf.grad.float(), xu.grad.float(), rtol=2e-2, atol=2e-3)
    # the fused reduce sums dp over the windows unrounded; the unfused one summed
    # dz rounded to bf16 where windows share a winning tap: norm-level agreement
    for a, r in ((bn_f.weight.grad, bn_u.weight.grad), (bn_f.bias.grad, bn_u.bias.grad)):
        assert float((a - r).norm() / (r.norm() + 1e-12)) < 5e-3

    # fp32 PyTorch reference
    xr = x0.detach().float().requires_grad_(True)
    g = make()
    w = g.weight.detach().float().requires_grad_(True)
    b = g.bias.detach().float().requires_grad_(True)
    yr = F.max_pool2d(F.relu(F.batch_norm(xr, None, None, w, b, True, 0.1, 1e-5)), 3, 2, 1)
    (yr * dp).sum().backward()
    torch.testing.assert_close(yf.float(), yr, rtol=2e-2, atol=2e-2)
    def rel(a, r):
        return float((a.float() - r).norm() / (r.norm() + 1e-12))

    assert rel(xf.grad, xr.grad) < 4e-2      # bf16 dz through a 25k-row BN reduction
    assert rel(bn_f.weight.grad, w.grad) < 1e-2
    assert rel(bn_f.bias.grad, b.grad) < 1e-2


@pytest.mark.parametrize("mode", ["elem", "nchw", "nhwc"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_dropout_kernel(mode, dtype):
    from distributed_ml_pytorch_amd.ops import layers as L

    torch.manual_seed(0)
    x = torch.randn(8, 32, 9, 9, device="cuda").to(dtype)
    if mode == "nhwc":
        x = x.contiguous(memory_format=torch.channels_last)
    layer = (L.Dropout(0.3, seed=7) if mode == "elem" else L.Dropout2d(0.3, seed=7)).cuda()
    x.requires_grad_(True)
    y = layer(x)
    keep = y.float() != 0
    frac = keep.float().mean().item()
    assert abs(frac - 0.7) < 0.03
    scale = 1.0 / 0.7
    torch.testing.assert_close(y.float()[keep], (x.detach().float() * scale)[keep],
                               rtol=1e-2, atol=1e-2)
    if mode != "elem":   # one draw per (n, c) plane
        per_plane = keep.float().mean(dim=(2, 3))
        assert bool(((per_plane == 0) | (per_plane == 1)).all())
    g = torch.randn_like(y)
    y.backward(g)
    torch.testing.assert_close(x.grad.float(), (g.float() * keep.float() * scale),
                               rtol=1e-2, atol=1e-2)
    # the device offset advances: a second call draws a different mask
    y2 = layer(x.detach())
    assert not torch.equal(y2 != 0, y != 0)
    # the fused kernel advanced its own offset (last block) and reset the ticket
    assert layer._state.tolist() == [2, 0]
    layer.eval()
    assert layer(x) is x


@pytest.mark.parametrize("rows,D", [(111, 768), (111, 192), (111, 4096), (111, 64), (37, 24),
                                    (12608, 768), (5000, 1024)])
def test_layernorm_kernel(rows, D):
    """Native LayerNorm fwd/bwd vs fp32 PyTorch; the persistent param-grad slot
    buffer must come back zeroed, so a second backward with it is exact too."""
    from distributed_ml_pytorch_amd.ops.functional import LN_SLOTS, layer_norm, layernorm_supported

    assert layernorm_supported(D)
    torch.manual_seed(0)
    slots = torch.zeros(LN_SLOTS * 2 * D, device="cuda")
    rel = lambda a, r: float((a.float() - r).norm() / r.norm())
    for _ in range(2):
        x = (torch.randn(rows, D, device="cuda") * 2 + 0.5).to(torch.bfloat16).requires_grad_(True)
        w = (1 + 0.1 * torch.randn(D, device="cuda")).requires_grad_(True)
        b = (0.1 * torch.randn(D, device="cuda")).requires_grad_(True)
        y = layer_norm(x, w, b, 1e-6, slots)
        xr = x.detach().float().requires_grad_(True)
        wr = w.detach().clone().requires_grad_(True)
        br = b.detach().clone().requires_grad_(True)
        yr = F.layer_norm(xr, (D,), wr, br, 1e-6)
        torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
        g = torch.randn_like(yr)
        y.backward(g.to(torch.bfloat16))
        yr.backward(g.to(torch.bfloat16).float())
        assert rel(x.grad, xr.grad) < 1e-2
        assert rel(w.grad, wr.grad) < 1e-2
        assert rel(b.grad, br.grad) < 1e-2
        assert float(slots.abs().max()) == 0.0


@pytest.mark.parametrize("rows,D,use_h", [(12608, 768, True), (394, 768, False), (37, 200, True)])
def test_add_layernorm_kernel(rows, D, use_h):
    """Fused residual add + LayerNorm: h = bf16(x + r), y = LN(h); the backward
    adds the residual stream's own gradient (dh) inside the LN-backward kernel."""
    from distributed_ml_pytorch_amd.ops.functional import LN_SLOTS, add_layer_norm

    torch.manual_seed(0)
    slots = torch.zeros(LN_SLOTS * 2 * D, device="cuda")
    rel = lambda a, r: float((a.float() - r).norm() / r.norm())
    x = torch.randn(rows, D, device="cuda").to(torch.bfloat16).requires_grad_(True)
    r = torch.randn(rows, D, device="cuda").to(torch.bfloat16).requires_grad_(True)
    w = (1 + 0.1 * torch.randn(D, device="cuda")).requires_grad_(True)
    b = (0.1 * torch.randn(D, device="cuda")).requires_grad_(True)
    h, y = add_layer_norm(x, r, w, b, 1e-6, slots)
    xr = x.detach().float().requires_grad_(True)
    rr = r.detach().float().requires_grad_(True)
    wr = w.detach().clone().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    hr = xr + rr
    yr = F.layer_norm(hr, (D,), wr, br, 1e-6)
    torch.testing.assert_close(h.float(), hr, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
    gy = torch.randn_like(yr).to(torch.bfloat16)
    gh = torch.randn_like(hr).to(torch.bfloat16)
    if use_h:
        torch.autograd.backward([y, h], [gy, gh])
        torch.autograd.backward([yr, hr], [gy.float(), gh.float()])
    else:
        y.backward(gy)
        yr.backward(gy.float())
    assert rel(x.grad, xr.grad) < 1e-2
    assert rel(r.grad, rr.grad) < 1e-2
    assert rel(w.grad, wr.grad) < 1e-2
    assert rel(b.grad, br.grad) < 1e-2
    assert float(slots.abs().max()) == 0.0


@pytest.mark.parametrize("M,N", [(12608, 768), (300, 3072), (7, 8), (1000, 4104)])
def test_colsum_acc(M, N):
    from distributed_ml_pytorch_amd.ops._ext import native

    torch.manual_seed(0)
    dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    out = torch.randn(N, device="cuda")
    ref = out + dy.float().sum(0)
    slots = torch.zeros(native().colsum_num_slots() * N, device="cuda")
    native().colsum_acc(dy, out, slots)
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-2)
    assert float(slots.abs().max()) == 0.0
    x4 = torch.randn(4, 64, 5, 7, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    o4 = torch.zeros(64, device="cuda")
    native().colsum_acc(x4, o4)
    torch.testing.assert_close(o4, x4.float().sum((0, 2, 3)), rtol=1e-4, atol=1e-2)


def test_gelu_kernel():
    from distributed_ml_pytorch_amd.ops.functional import gelu

    x = (torch.randn(64, 3072, device="cuda") * 3).to(torch.bfloat16).requires_grad_(True)
    y = gelu(x)
    xr = x.detach().float().requires_grad_(True)
    yr = F.gelu(xr, approximate="tanh")
    torch.testing.assert_close(y.float(), yr, rtol=1e-2, atol=1e-2)
    g = torch.randn_like(yr).to(torch.bfloat16)
    y.backward(g)
    yr.backward(g.float())
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("N", [197, 65, 1000])
def test_attention_softmax(N):
    from distributed_ml_pytorch_amd.ops.functional import attention

    torch.manual_seed(0)
    q, k, v = (torch.randn(2, 3, N, 64, device="cuda").to(torch.bfloat16).requires_grad_(True)
               for _ in range(3))
    o = attention(q, k, v)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    orf = F.scaled_dot_product_attention(qr, kr, vr)
    rel = lambda a, r: float((a.float() - r).norm() / r.norm())
    assert rel(o, orf) < 2e-2
    g = torch.randn_like(orf)
    o.backward(g.to(torch.bfloat16))
    orf.backward(g.to(torch.bfloat16).float())
    for a, r in ((q, qr), (k, kr), (v, vr)):
        assert rel(a.grad, r.grad) < 3e-2


@pytest.mark.parametrize("B,N,H", [(2, 197, 12), (3, 65, 2), (1, 256, 1), (2, 5, 3), (4, 32, 4)])
def test_fused_qkv_attention(B, N, H):
    """csrc/attention.hip fwd + bwd vs fp32 SDPA on the same qkv rows."""
    from distributed_ml_pytorch_amd.ops.functional import attention_qkv, fused_attention_supported

    torch.manual_seed(0)
    D = 64 * H
    qkv = torch.randn(B, N, 3 * D, device="cuda").to(torch.bfloat16).requires_grad_(True)
    assert fused_attention_supported(qkv, H)
    o = attention_qkv(qkv, H)
    qr = qkv.detach().float().requires_grad_(True)
    q, k, v = qr.view(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
    orf = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, N, D)
    rel = lambda a, r: float((a.float() - r).norm() / r.norm())
    assert o.shape == (B, N, D)
    assert rel(o, orf) < 1e-2, rel(o, orf)
    g = torch.randn_like(orf).to(torch.bfloat16)
    o.backward(g)
    orf.backward(g.float())
    for t in range(3):
        a = qkv.grad.view(B, N, 3, D)[:, :, t]
        r = qr.grad.view(B, N, 3, D)[:, :, t]
        assert rel(a, r) < 2e-2, (t, rel(a, r))


@pytest.mark.parametrize("C", [10, 1000])
def test_xent_ignore_index_grad_is_mean_over_valid_rows(C):
    """Rows labelled ignore_index (and out-of-range labels) contribute nothing and
    the gradient is scaled by 1/#valid, matching F.cross_entropy's mean."""
    from distributed_ml_pytorch_amd.ops.functional import softmax_cross_entropy

    torch.manual_seed(0)
    B = 300
    x = torch.randn(B, C, device="cuda").to(torch.bfloat16).requires_grad_(True)
    y = torch.randint(0, C, (B,), device="cuda")
    y[::3] = -100
    loss, hits = softmax_cross_entropy(x, y)
    loss.backward()
    xr = x.detach().float().requires_grad_(True)
    lr = torch.nn.functional.cross_entropy(xr, y, ignore_index=-100)
    lr.backward()
    torch.testing.assert_close(loss.float(), lr, rtol=1e-2, atol=1e-3)
    assert float((x.grad.float() - xr.grad).norm() / xr.grad.norm()) < 1e-2
    assert float(x.grad[::3].float().abs().max()) == 0.0


def test_relu_mask_hand_off_with_two_consumers():
    """A fused-ReLU conv output feeding BOTH a max-pool (whose backward marks its
    gradient as already relu'-masked) and a second consumer: autograd sums the
    two gradients (possibly in place into the pool's tensor), so the conv must
    mask the SUM.  Compared against fp32 PyTorch."""
    import torch.nn.functional as F

    from distributed_ml_pytorch_amd.ops.functional import max_pool2d
    from distributed_ml_pytorch_amd.ops.layers import Conv2d

    torch.manual_seed(0)
    conv = Conv2d(64, 64, 3, padding=1, bias=False).cuda()
    x = torch.randn(4, 64, 16, 16, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    c = torch.randn(4, 64, 16, 16, device="cuda")
    ga = torch.randn(4, 64, 8, 8, device="cuda")
    for order in ("pool_first", "mul_first"):
        conv.weight.grad = None
        y = conv(x, relu=True)
        if order == "pool_first":
            loss = (max_pool2d(y, 2).float() * ga).sum() + (y.float() * c).sum()
        else:
            loss = (y.float() * c).sum() + (max_pool2d(y, 2).float() * ga).sum()
        loss.backward()
        wr = conv.weight.detach().to(torch.bfloat16).float().requires_grad_(True)
        yr = F.relu(F.conv2d(x.float(), wr, None, 1, 1))
        lr = (F.max_pool2d(yr, 2) * ga).sum() + (yr * c).sum()
        lr.backward()
        rel = float((conv.weight.grad - wr.grad).norm() / wr.grad.norm())
        # bf16 outputs move a few max-pool argmaxes (near-ties): a few % of noise;
        # a skipped ReLU mask on the summed gradient is an O(1) error
        assert rel < 5e-2, (order, rel)


@pytest.mark.parametrize("B,C,H,N", [(512, 512, 4, 10), (37, 2048, 7, 16), (5, 64, 8, 3), (9, 1024, 2, 7), (3, 1000, 2, 7)])
def test_gap_linear_head_fused(B, C, H, N):
    """Fused global-average-pool + Linear head (csrc/head.hip): logits, dx, dW (+=)
    and db (+=) against fp32 autograd of mean-pool + linear."""
    from distributed_ml_pytorch_amd.ops._ext import native

    nat = native()
    if not nat.gap_linear_supported(C, N):
        pytest.skip("geometry outside the fused head")
    torch.manual_seed(0)
    x = torch.randn(B, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(N, C, device="cuda") / C ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device="cuda").to(torch.bfloat16)
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    br = b.float().requires_grad_(True)
    yr = torch.nn.functional.linear(xr.mean(dim=(2, 3)), wr, br)
    dy = torch.randn(B, N, device="cuda").to(torch.bfloat16)
    yr.backward(dy.float())
    y, f = nat.gap_linear_fwd(x, w, b)
    assert float((y.float() - yr).norm() / yr.norm()) < 1e-2
    gw = torch.full((N, C), 0.5, device="cuda")
    gb = torch.full((N,), 0.25, device="cuda")
    dx = nat.gap_linear_bwd(dy, f, w, gw, gb, H, H)
    assert dx.is_contiguous(memory_format=torch.channels_last) and dx.shape == x.shape
    assert float((dx.float() - xr.grad).norm() / xr.grad.norm()) < 1e-2
    assert float((gw - 0.5 - wr.grad).norm() / wr.grad.norm()) < 1e-2
    assert float((gb - 0.25 - br.grad).norm() / br.grad.norm()) < 1e-2


@pytest.mark.parametrize("B,C,H,mode", [(64, 64, 32, 2), (32, 64, 32, 3), (64, 256, 8, 3),
                                        (16, 512, 4, 0), (3, 80, 7, 2)])
def test_bn_bwd_onepass(B, C, H, mode):
    """One-launch BatchNorm backward (bn.hip bn_bwd_onepass_kernel: reduce ->
    last-arriver coefficient fold -> apply on the same rows) at ResNet-18 sizes,
    ReLU mask from x (mode 2), from the 1-bit mask (mode 3) or none, vs fp32; the
    slot buffer's hand-off words are re-armed (zero) after every call and the
    bounded poll never gave up; dgamma / dbeta accumulate across calls."""
    from distributed_ml_pytorch_amd.ops._ext import native

    nat = native()
    torch.manual_seed(B + C)
    M = B * H * H
    x = _bf(torch.randn(B, C, H, H, device="cuda") * 1.5 + 0.3).contiguous(memory_format=CL)
    dy = _bf(torch.randn(B, C, H, H, device="cuda")).contiguous(memory_format=CL)
    gamma = torch.rand(C, device="cuda") + 0.5
    beta = torch.randn(C, device="cuda") * 0.2
    xf = x.float()
    mean = xf.mean(dim=(0, 2, 3))
    var = xf.var(dim=(0, 2, 3), unbiased=False)
    inv = torch.rsqrt(var + 1e-5)
    sc, sh = gamma * inv, beta - mean * gamma * inv
    stats = torch.cat([mean, inv, sc, sh]).contiguous()
    pre = xf * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1)
    mask = None
    if mode == 0:
        on = torch.ones_like(pre, dtype=torch.bool)
    elif mode == 2:
        on = _bf(torch.relu(pre)).float() > 0
    else:
        on = torch.rand_like(pre) > 0.4
        bits = on.permute(0, 2, 3, 1).reshape(-1, 8).to(torch.uint8)
        mask = (bits << torch.arange(8, device="cuda", dtype=torch.uint8)).sum(1).to(torch.uint8)
    dz = torch.where(on, dy.float(), torch.zeros(()))
    xhat = (xf - mean.view(1, -1, 1, 1)) * inv.view(1, -1, 1, 1)
    db_ref = dz.sum(dim=(0, 2, 3))
    dg_ref = (dz * xhat).sum(dim=(0, 2, 3))
    dx_ref = (gamma * inv).view(1, -1, 1, 1) * (dz - db_ref.view(1, -1, 1, 1) / M
                                                 - xhat * dg_ref.view(1, -1, 1, 1) / M)
    slots = torch.zeros(2 * 64 * C + 4, device="cuda")
    fwd_slots = torch.ones(2 * 64 * C + 4, device="cuda")
    dgam = torch.zeros(C, device="cuda")
    dbet = torch.zeros(C, device="cuda")
    for it in range(3):
        dx, _ = nat.bn_bwd_fold(x, dy, None, gamma, stats, dgam, dbet, mode != 0, False, slots,
                                mask, fwd_slots)
        torch.cuda.synchronize()
        tail = slots[-4:].view(torch.int32)
        assert tail.tolist() == [0, 0, 0, 0], tail.tolist()
        assert torch.count_nonzero(fwd_slots[:-4]) == 0          # forward slots zeroed
        torch.testing.assert_close(dx.float(), dx_ref, rtol=3e-2, atol=3e-2)
        torch.testing.assert_close(dbet, (it + 1) * db_ref, rtol=1e-3, atol=1e-2 * (it + 1))
        torch.testing.assert_close(dgam, (it + 1) * dg_ref, rtol=1e-3, atol=1e-2 * (it + 1))
        slots[:-4].zero_()    # (the next forward apply re-zeroes these in a model)
