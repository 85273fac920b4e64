"""BatchNorm(+ReLU) backward of the native kernels vs fp32 torch, per component."""
import sys

import torch
import torch.nn.functional as TF

sys.path.insert(0, ".")
from deep_vision_amd import nn, ops as F  # noqa: E402

DEV = "cuda"


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


for C, H, N in ((32, 112, 64), (512, 14, 64), (64, 56, 32)):
    for act in (None, "relu"):
        torch.manual_seed(0)
        bn = nn.BatchNorm2d(C).to(DEV)
        bn.weight.data.uniform_(0.5, 1.5)
        bn.bias.data.uniform_(-0.3, 0.3)
        x32 = torch.randn(N, C, H, H, device=DEV).bfloat16().float()
        x = x32.to(torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_(True)
        y = F.batch_norm_act(x, bn, act)
        dy = torch.randn(y.shape, device=DEV).bfloat16().float()
        y.backward(dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
        w = bn.weight.detach().clone().requires_grad_(True)
        b = bn.bias.detach().clone().requires_grad_(True)
        xr = x32.clone().requires_grad_(True)
        yr = TF.batch_norm(xr, None, None, w, b, True, 0.1, bn.eps)
        if act:
            yr = TF.relu(yr)
        yr.backward(dy)
        mm = ((y.float() > 0) != (yr > 0)).float().mean().item() if act else 0.0
        # exact dx from torch formula on the native forward's own z, for comparison
        print(f"C{C}@{H} N{N} act={act}: y {rel(y, yr):.2e} maskflip {mm:.2e} dx {rel(x.grad, xr.grad):.2e} "
              f"dgamma {rel(bn.weight.grad, w.grad):.2e} dbeta {rel(bn.bias.grad, b.grad):.2e}", flush=True)
