"""Stem conv (7x7 s2, 3 -> 64, batch 256 @ 224) forward / wgrad time per packed-kernel variant.
usage: python tools/stem_bench.py"""
import sys

import torch

sys.path.insert(0, ".")
from deep_vision_amd import ops as F  # noqa: E402
from deep_vision_amd._ext import lib  # noqa: E402

x = torch.randn(256, 3, 224, 224, device="cuda")
w = (torch.randn(64, 3, 7, 7, device="cuda") * 0.05).requires_grad_(True)
for v in (0, 5, 7, 8, 0):
    lib().conv_fwd_variant(v)
    for _ in range(3):
        y = F.conv2d(x, w, None, 2, 3)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    e[0].record()
    for _ in range(10):
        y = F.conv2d(x, w, None, 2, 3)
    e[1].record()
    g = torch.randn_like(y)
    for _ in range(10):
        w.grad = None
        torch.autograd.grad(F.conv2d(x, w, None, 2, 3), w, g)
    e[2].record()
    torch.cuda.synchronize()
    f = e[0].elapsed_time(e[1]) / 10 * 1e3
    fb = e[1].elapsed_time(e[2]) / 10 * 1e3
    print(f"variant {v}: fwd (incl. pack) {f:7.1f} us   fwd+wgrad {fb:7.1f} us", flush=True)
lib().conv_fwd_variant(0)
