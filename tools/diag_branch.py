"""Hourglass training trajectories (6 SGD steps) under: eager single stream, eager forked branch
streams, captured without forking, captured with forking."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_vision_amd.models import hourglass as H  # noqa: E402
from deep_vision_amd.ops.loss import heatmap_mse  # noqa: E402
from deep_vision_amd.train.graph import CapturedStep  # noqa: E402
from deep_vision_amd.train.optim import FusedSGD  # noqa: E402

torch.manual_seed(0)
base = H.StackedHourglassNetwork(num_stack=2, num_residual=1, num_heatmap=16).cuda()
xs = [torch.randn(4, 3, 128, 128, device="cuda") for _ in range(6)]
hms = [torch.rand(4, 16, 32, 32, device="cuda") for _ in range(6)]


def make(model, opt):
    def step(x, hm):
        opt.zero_grad()
        loss = sum(heatmap_mse(y, hm) for y in model(x))
        loss.backward()
        opt.step()
        return loss
    return step


def eager(fork):
    H.BRANCH_STREAMS = fork
    m = copy.deepcopy(base)
    st = make(m, FusedSGD(m.parameters(), lr=1e-4))
    return [round(st(xs[i], hms[i]).item(), 4) for i in range(6)]


def captured(mode):
    H.BRANCH_STREAMS = mode
    m = copy.deepcopy(base)
    o = FusedSGD(m.parameters(), lr=1e-4)
    sb = make(m, o)
    warm = iter([(xs[0], hms[0]), (xs[1], hms[1])])
    out = []

    def fn(x, hm):
        w = next(warm, None)
        if w is not None:
            x.copy_(w[0])
            hm.copy_(w[1])
        loss = sb(x, hm)
        return loss

    cap = CapturedStep(fn, o, (xs[0].clone(), hms[0].clone()), model=m, warmup=2)
    out.append(round(cap.warmup_outputs.item(), 4))
    for i in range(2, 6):
        out.append(round(cap(xs[i], hms[i]).item(), 4))
    return out


print("eager single   ", eager(False))
print("eager forked   ", eager(True))
print("eager single   ", eager(False))
print("captured nofork", captured(False))
print("captured fork  ", captured("graph"))
