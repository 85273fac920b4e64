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
        return lr.mean()  # one reduction launch (sum and scale fused)

    @staticmethod
    def backward(ctx, go):
        (grad,) = ctx.saved_tensors
        if go is None:
            return grad, None, None
        # out of place: the saved buffer stays the unscaled gradient, so a second backward through
        # a retained graph scales the same values again (an in-place mul_ would have returned
        # grad*go1*go2); the scale is read on the device by one native launch
        go = go.detach().to(F32).reshape(1).contiguous()
        out = torch.empty_like(grad)
        lib().scale_by(ptr(grad), ptr(out), grad.numel(), int(grad.dtype == BF16), ptr(go), stream_handle())
        return out, None, None


def cross_entropy(logits, labels, label_smoothing=0.0):
    if not native(logits):
        return TF.cross_entropy(logits, labels, label_smoothing=label_smoothing)
    if logits.dtype not in (BF16, F32) or not logits.is_contiguous():
        logits = logits.contiguous()
        if logits.dtype not in (BF16, F32):
            logits = logits.float()
    labels = labels.contiguous().long()
    return _XentFn.apply(logits, labels, float(label_smoothing))


# ------------------------------------------------------------------------------------------
# Pointwise losses (csrc/losses.hip): one pass computes the sum, the backward launch writes the
# gradient scaled by the upstream gradient read from device memory (no host synchronisation).
# ------------------------------------------------------------------------------------------
_KINDS = {"wmse": 0, "mse": 1, "l1": 2, "bce_logits": 3, "focal": 4}


def _rows(x):
    """(rows, C, ld) of the physical layout of ``x`` (NHWC 4-D or contiguous)."""
    from .common import is_nhwc, ld_of

    if x.dim() == 4 and is_nhwc(x):
        N, C, H, W = x.shape
        return N * H * W, C, ld_of(x)
    return x.numel(), 1, 1


def _native_pred(x):
    from .common import is_nhwc

    if x.dim() == 4 and is_nhwc(x):
        return x
    if x.dtype in (BF16, F32) and x.is_contiguous():
        return x
    if x.dim() == 4:
        return x.to(BF16).contiguous(memory_format=torch.channels_last)
    return x.contiguous()


def _match_target(t, pred):
    if pred.dim() == 4 and pred.stride(1) == 1 and pred.shape[1] > 1:
        t = t.contiguous(memory_format=torch.channels_last)
    else:
        t = t.contiguous()
    if t.dtype not in (BF16, F32):
        t = t.float()
    return t, (1 if t.dtype == BF16 else 0)


class _PWLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target, tval, kind, a, b, norm, weight=None):
        rows, C, ld = _rows(pred)
        dev = pred.device
        sums = torch.zeros(2, dtype=F32, device=dev)
        if target is not None:
            target, ttype = _match_target(target, pred)
        else:
            ttype = 2
        if weight is not None:
            weight = _match_target(weight.float(), pred)[0]
        lib().pw_loss(kind, ptr(pred), int(pred.dtype == BF16), ptr(target), ttype, float(tval), ptr(weight), rows, C,
                      ld, C, a, b, ptr(sums), 0, 0, 1.0, stream_handle())
        if kind == _KINDS["focal"]:
            scale = 1.0 / sums[1].clamp(min=1.0)
        else:
            scale = torch.full((), norm, dtype=F32, device=dev)
        ctx.save_for_backward(pred, target, scale, weight)
        ctx.cfg = (tval, kind, a, b, ttype)
        return sums[0] * scale

    @staticmethod
    def backward(ctx, gout):
        pred, target, scale, weight = ctx.saved_tensors
        tval, kind, a, b, ttype = ctx.cfg
        rows, C, ld = _rows(pred)
        gs = (gout.float() * scale).reshape(1).contiguous()
        if pred.dim() == 4 and ld != pred.shape[1]:
            from .common import empty_nhwc

            grad = empty_nhwc(*pred.shape, pred.device)
        else:
            grad = torch.empty_like(pred)
        lib().pw_loss(kind, ptr(pred), int(pred.dtype == BF16), ptr(target), ttype, float(tval), ptr(weight), rows, C,
                      ld, C, a, b, 0, ptr(grad), ptr(gs), 1.0, stream_handle())
        return grad, None, None, None, None, None, None, None


def _pw(pred, target, kind, a=0.0, b=0.0, reduction="mean", weight=None, norm=None):
    if isinstance(target, (int, float)):
        tval, target_t = float(target), None
    else:
        tval, target_t = 0.0, target
    if weight is not None and target_t is None:
        target_t = torch.full(pred.shape, tval, dtype=F32, device=pred.device)
    pred = _native_pred(pred)
    if norm is None:
        norm = 1.0 / pred.numel() if reduction == "mean" else 1.0
    return _PWLossFn.apply(pred, target_t, tval, _KINDS[kind], float(a), float(b), norm, weight)


def _full_like(t, v):
    return torch.full_like(t, v) if isinstance(v, (int, float)) else v


def heatmap_mse(pred, target, fg_weight=81.0):
    """mean((t - p)^2 * (1 + fg_weight [t > 0])) -- the Hourglass loss of one stack
    (R/Hourglass/tensorflow/train.py:65-76; the trainer divides by the global batch)."""
    if not native(pred):
        w = (target > 0).float() * fg_weight + 1
        return ((target - pred.float()) ** 2 * w).mean()
    return _pw(pred, target, "wmse", a=fg_weight)


def mse_loss(pred, target, reduction="mean"):
    """MSE against a tensor or a constant label (LSGAN, R/CycleGAN/tensorflow/train.py:53-62)."""
    if not native(pred):
        d = (pred.float() - _full_like(pred.float(), target)) ** 2
        return d.mean() if reduction == "mean" else d.sum()
    return _pw(pred, target, "mse", reduction=reduction)


def l1_loss(pred, target, reduction="mean"):
    if not native(pred):
        d = (pred.float() - _full_like(pred.float(), target).float()).abs()
        return d.mean() if reduction == "mean" else d.sum()
    return _pw(pred, target, "l1", reduction=reduction)


def bce_with_logits(logits, target, reduction="mean"):
    """tf.keras.losses.BinaryCrossentropy(from_logits=True) (R/DCGAN/tensorflow/main.py:42-53)."""
    if not native(logits):
        return TF.binary_cross_entropy_with_logits(logits.float(), _full_like(logits.float(), target).float(),
                                                   reduction=reduction)
    return _pw(logits, target, "bce_logits", reduction=reduction)


def focal_loss(logits, target, alpha=2.0, beta=4.0):
    """CenterNet penalty-reduced pixel-wise focal loss on sigmoid(logits), normalised by the number
    of positive (t == 1) locations."""
    if not native(logits):
        p = torch.sigmoid(logits.float()).clamp(1e-4, 1 - 1e-4)
        t = target.float()
        pos = t.ge(1).float()
        lp = -((1 - p) ** alpha) * torch.log(p) * pos
        ln = -((1 - t) ** beta) * p ** alpha * torch.log(1 - p) * (1 - pos)
        return (lp.sum() + ln.sum()) / pos.sum().clamp(min=1)
    return _pw(logits, target, "focal", a=alpha, b=beta, reduction="sum")


def masked_l1(pred, target, mask, num=None):
    """sum(|p - t| * mask) / max(num, 1) -- CenterNet size / offset regression at object centres
    (``mask`` in the target's shape; ``num`` a host count, default ``mask.sum()`` synced)."""
    n = float(max(1.0, float(mask.sum()) if num is None else num))
    if not native(pred):
        return ((pred.float() - target.float()).abs() * mask.float()).sum() / n
    return _pw(pred, target, "l1", weight=mask, norm=1.0 / n)
