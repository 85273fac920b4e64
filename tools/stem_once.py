"""One stem conv forward + weight gradient at the ResNet-50 shape (batch 256, 224x224, 7x7/2,
3 -> 64) for rocprofv3 PMC passes: python tools/stem_once.py [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_vision_amd import ops as F  # noqa: E402

it = int(sys.argv[1]) if len(sys.argv) > 1 else 2
x = torch.randn(256, 3, 224, 224, device="cuda")
w = (torch.randn(64, 3, 7, 7, device="cuda") * 0.05).requires_grad_(True)
for _ in range(it):
    y = F.conv2d(x, w, None, 2, 3)
    g = torch.randn_like(y)
    torch.autograd.grad(y, w, g)
torch.cuda.synchronize()
