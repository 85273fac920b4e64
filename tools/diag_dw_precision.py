"""Gradient deviation from fp32 of depthwise conv / BN+ReLU / both, native vs autocast bf16."""
import copy
import sys

import torch
import torch.nn.functional as TF

sys.path.insert(0, ".")
from deep_vision_amd import nn, ops as F  # noqa: E402

DEV = "cuda"


def cosd(a, b):
    a, b = a.float().flatten(), b.float().flatten()
    return 1 - (a @ b / (a.norm() * b.norm())).item()


class M(torch.nn.Module):
    def __init__(self, C, s, use_dw, use_bn, pw=False):
        super().__init__()
        self.use_dw, self.use_bn = use_dw, use_bn
        self.dw = nn.Conv2d(C, C, 3, stride=s, padding=1, groups=C, bias=False) if not pw else nn.Conv2d(C, C, 1, bias=False)
        self.bn = nn.BatchNorm2d(C)

    def forward(self, x):
        if self.use_dw and self.use_bn:
            return F.conv_bn_act(x, self.dw, self.bn, "relu")
        if self.use_dw:
            return self.dw(x)
        return F.batch_norm_act(x, self.bn, "relu") if F.native(x) else TF.relu(self.bn(x))


for C, H, s in ((32, 112, 1), (512, 14, 1)):
    for name, dw, bn, pw in (("dw", 1, 0, 0), ("bnrelu", 0, 1, 0), ("dw+bnrelu", 1, 1, 0), ("pw+bnrelu", 1, 1, 1)):
        torch.manual_seed(0)
        m = M(C, s, dw, bn, pw).to(DEV)
        m.bn.weight.data.uniform_(0.5, 1.5)
        m.bn.bias.data.uniform_(-0.3, 0.3)
        x32 = torch.randn(64, C, H, H, device=DEV).bfloat16().float()
        x = x32.to(torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_(True)
        y = m(x)
        dy = torch.randn(y.shape, device=DEV).bfloat16().float()
        y.backward(dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
        res = {}
        for ac in (False, True):
            r = copy.deepcopy(m).float()
            for p in r.parameters():
                p.data.copy_(p.data.bfloat16().float())
                p.grad = None
            xr = x32.clone().requires_grad_(True)
            F.set_backend("torch")
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=ac):
                yr = r(xr)
            yr.float().backward(dy)
            F.set_backend("native")
            res[ac] = (xr.grad, yr.float(), [p.grad for p in r.parameters() if p.grad is not None])
        g32, y32, p32 = res[False]
        gb, yb, pb = res[True]
        pn = [p.grad for p in m.parameters() if p.grad is not None]
        print(f"C{C}@{H} {name:10s} fwd native {cosd(y, y32):.2e} ac {cosd(yb, y32):.2e} | dx native {cosd(x.grad, g32):.2e} "
              f"ac {cosd(gb, g32):.2e} | params native {[f'{cosd(a, b):.1e}' for a, b in zip(pn, p32)]} "
              f"ac {[f'{cosd(a, b):.1e}' for a, b in zip(pb, p32)]}", flush=True)
