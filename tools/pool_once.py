"""One fused BN -> ReLU -> max-pool forward + backward at the ResNet-50 stem shape (batch 256,
64 x 112 x 112) for rocprofv3 runs: python tools/pool_once.py [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_vision_amd import nn  # noqa: E402
from deep_vision_amd import ops as F  # noqa: E402

it = int(sys.argv[1]) if len(sys.argv) > 1 else 2
bn = nn.BatchNorm2d(64).cuda()
pool = nn.MaxPool2d(3, 2, 1)
x = torch.randn(256, 64, 112, 112, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
x.requires_grad_(True)
for _ in range(it):
    y = F.batch_norm_act_maxpool(x, bn, "relu", 0.0, pool)
    y.backward(torch.ones_like(y))
torch.cuda.synchronize()
