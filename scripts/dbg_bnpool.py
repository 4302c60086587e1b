"""Debug: fused BN+ReLU+pool backward reduce vs a PyTorch recomputation from xm / idx / dp."""
import torch
from distributed_ml_pytorch_amd.ops._ext import native
CL = torch.channels_last
torch.manual_seed(1)
N, C, H, W = 4, 64, 16, 16
x = (torch.randn(N, C, H, W, device="cuda") * 2 + 0.3).to(torch.bfloat16).contiguous(memory_format=CL)
g = (torch.rand(C) + 0.5).cuda(); g[::7] *= -1
b = (torch.randn(C) * 0.2).cuda()
fs = torch.zeros(2 * 64 * C + 4, device="cuda"); bs = torch.zeros_like(fs)
y, idx, stats, xm = native().bn_relu_maxpool_fwd(x, fs, False, g, b, None, None, 0.1, 1e-5, bs, 3, 2, 1)
torch.cuda.synchronize()
mean, inv = stats[0], stats[1]
xf = x.float()
# reference: pool over relu(bn(x)) in fp32 with the same rounding
yy = torch.relu(xf * stats[2].view(1, C, 1, 1) + stats[3].view(1, C, 1, 1)).to(torch.bfloat16).float()
yr, ir = torch.nn.functional.max_pool2d(yy, 3, 2, 1, return_indices=True)
print("y equal", torch.equal(y.float(), yr))
xr = xf.flatten(2).gather(2, ir.flatten(2)).view_as(yr)
valid = yr > 0
print("xm match (valid)", float(((xm.float() - xr).abs() * valid).max()))
dp = torch.randn_like(yr).to(torch.bfloat16).float()
dz_sum = (dp * valid).sum((0, 2, 3))
dzx = (dp * valid * (xr - mean.view(1, C, 1, 1)) * inv.view(1, C, 1, 1)).sum((0, 2, 3))
dg = torch.zeros(C, device="cuda"); db = torch.zeros(C, device="cuda")
slots = torch.zeros_like(fs)
dx = native().maxpool_bn_bwd(x, dp.to(torch.bfloat16).contiguous(memory_format=CL), idx, xm, g, stats, dg, db, slots, fs, 3, 2, 1)
torch.cuda.synchronize()
print("db", float((db - dz_sum).abs().max()), float(dz_sum.abs().max()))
print("dg", float((dg - dzx).abs().max()), float(dzx.abs().max()))
print("idx sample", idx.flatten()[:16].tolist())

# the test's flow: module-level fused vs unfused
from distributed_ml_pytorch_amd.ops import functional as DF
from distributed_ml_pytorch_amd.ops import layers as L
def make():
    bn = L.BatchNorm2d(C, relu=True).cuda()
    with torch.no_grad():
        bn.weight.copy_(g); bn.bias.copy_(b)
    return bn
bn_f, bn_u = make(), make()
xf1 = x.clone().requires_grad_(True)
yf = DF.bn_relu_maxpool(xf1, bn_f, 3, 2, 1)
(yf.float() * dp).sum().backward()
DF._BN_POOL_FUSE = False
xu1 = x.clone().requires_grad_(True)
yu = DF.max_pool2d(bn_u(xu1), 3, 2, 1)
(yu.float() * dp).sum().backward()
torch.cuda.synchronize()
print("module fused dg vs exact", float((bn_f.weight.grad - dzx).abs().max()))
print("module unfused dg vs exact", float((bn_u.weight.grad - dzx).abs().max()))
print("module fused db vs exact", float((bn_f.bias.grad - dz_sum).abs().max()))
print("module unfused db vs exact", float((bn_u.bias.grad - dz_sum).abs().max()))
print("dx fused vs unfused", float((xf1.grad.float() - xu1.grad.float()).abs().max()))
