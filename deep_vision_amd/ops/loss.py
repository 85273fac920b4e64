"""Fused softmax cross-entropy (csrc/loss_optim.hip).

Matches ``nn.CrossEntropyLoss()`` (mean reduction) used by every PT classifier of the
reference (R/ResNet/pytorch/train.py:358). The gradient is produced in the forward launch.
"""
from __future__ import annotations

import torch
import torch.nn.functional as TF

from .common import BF16, F32, lib, native, ptr, stream_handle


class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, label_smoothing):
        B, C = logits.shape
        lr = torch.empty(B, dtype=F32, device=logits.device)
        need_grad = logits.requires_grad
        grad = torch.empty_like(logits) if need_grad else None
        lib().softmax_xent(ptr(logits), int(logits.dtype == BF16), ptr(labels), B, C, ptr(lr), ptr(grad), 1.0 / B,
                           float(label_smoothing), stream_handle())
        ctx.save_for_backward(grad)
        return lr.sum() / B

    @staticmethod
    def backward(ctx, go):
        (grad,) = ctx.saved_tensors
        g = grad if go is None else grad * go.to(grad.dtype)
        return g, None, None


def cross_entropy(logits, labels, label_smoothing=0.0):
    if not native(logits):
        return TF.cross_entropy(logits, labels, label_smoothing=label_smoothing)
    if logits.dtype not in (BF16, F32) or not logits.is_contiguous():
        logits = logits.contiguous()
        if logits.dtype not in (BF16, F32):
            logits = logits.float()
    labels = labels.contiguous().long()
    return _XentFn.apply(logits, labels, float(label_smoothing))
