"""Debug: conv producer -> folded BN, per-iteration error vs fp32."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_ml_pytorch_amd.ops import layers as L  # noqa: E402

CL = torch.channels_last
for C, H in ((64, 12), (128, 12), (64, 32)):
    torch.manual_seed(3)
    conv = L.Conv2d(64, C, 3, padding=1, bias=False).cuda()
    conv.emit_bn_stats = True
    bn = L.BatchNorm2d(C, relu=True).cuda()
    w16 = conv.weight.detach().to(torch.bfloat16).float()
    for it in range(4):
        x = torch.randn(8, 64, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        h = conv(x)
        part = h._dmp_bn_part
        ps = part[:2 * 64 * C].view(2, 64, C).sum(1)
        hf = h.float()
        e_s = float((ps[0] - hf.sum(dim=(0, 2, 3))).abs().max())
        e_q = float((ps[1] - (hf * hf).sum(dim=(0, 2, 3))).abs().max())
        y = bn(h)
        hr = F.conv2d(x.float(), w16, padding=1)
        yr = F.relu(F.batch_norm(hr, None, None, bn.weight.detach(), bn.bias.detach(), True))
        yh = F.relu(F.batch_norm(hf, None, None, bn.weight.detach(), bn.bias.detach(), True))
        print(f"C={C} H={H} it={it} slot-sum err {e_s:.3g}/{e_q:.3g} |y-yr| {float((y.float()-yr).abs().max()):.3g}"
              f" |y-yh| {float((y.float()-yh).abs().max()):.3g} |h-hr| {float((hf-hr).abs().max()):.3g}", flush=True)
        if it != 1:
            y.float().sum().backward()
