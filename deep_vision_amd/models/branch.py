"""Stream fork / join edge shared by the models that run independent branches on side HIP streams
(models/hourglass.py level branches, models/yolov3.py detector heads)."""
from __future__ import annotations

import torch


class BranchEdge(torch.autograd.Function):
    """Identity at a stream fork / join. Its backward runs on the branch's stream (autograd runs a
    node's backward on its forward stream) and marks the gradient crossing the edge as used by
    both streams: a gradient allocated on one stream and read on the other would otherwise go
    back to its allocating stream's pool while the other stream may still read it."""

    @staticmethod
    def forward(ctx, t, other):
        ctx.other = other
        return t.view_as(t)

    @staticmethod
    def backward(ctx, g):
        if g is not None:
            g.record_stream(torch.cuda.current_stream(g.device))
            g.record_stream(ctx.other)
        return g, None
