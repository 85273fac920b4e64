"""Flat parameter / gradient storage shared by the data-parallel layer and fused optimizers.

``flatten_parameters(model)`` moves every trainable parameter into ONE contiguous fp32 buffer
and every ``.grad`` into a matching flat gradient buffer (both as views). Parameters are laid
out in REVERSE registration order: autograd produces gradients roughly in reverse forward
order, so gradient buckets — plain slices of the flat gradient buffer — fill front to back
and can be all-reduced in place as soon as they are complete (no bucket copies).
"""
from __future__ import annotations

import torch


def flatten_parameters(model: torch.nn.Module, reverse: bool = True):
    params = [p for p in model.parameters() if p.requires_grad]
    if not params:
        raise ValueError("model has no trainable parameters")
    dev = params[0].device
    order = list(reversed(params)) if reverse else params
    total = sum(p.numel() for p in order)
    pflat = torch.empty(total, dtype=torch.float32, device=dev)
    gflat = torch.zeros(total, dtype=torch.float32, device=dev)
    off = 0
    layout = []
    shared = (pflat, gflat)  # one object: the optimizer recognises the layout by identity
    with torch.no_grad():
        for p in order:
            n = p.numel()
            pflat[off:off + n].view_as(p).copy_(p.data)
            p.data = pflat[off:off + n].view(p.shape)
            p.grad = gflat[off:off + n].view(p.shape)
            p._dv_flat = shared
            p._dv_off = off
            layout.append((p, off, n))
            off += n
    return pflat, gflat, layout
