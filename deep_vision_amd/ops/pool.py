"""Pooling and nearest upsampling on the native NHWC kernels (csrc/pool.hip).

Semantics follow torch.nn.MaxPool2d / AvgPool2d / AdaptiveAvgPool2d((1,1)) / Upsample as used
by the reference (e.g. R/ResNet/pytorch/models/resnet50.py:35 maxpool 3x3 s2 p1,
R/Inception/pytorch/models/inception_v1.py:29 ceil_mode maxpool, resnet50.py:45 GAP) and Keras
UpSampling2D(2) (R/YOLO/tensorflow/yolov3.py:151, R/Hourglass/tensorflow/hourglass104.py:96).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as TF

from .common import BF16, CL, as_nhwc, grad_nhwc, ld_of, lib, native, ptr, stream_handle, unsupported


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


def pool_out(H, k, s, p, ceil_mode, d=1):
    num = H + 2 * p - d * (k - 1) - 1
    if ceil_mode:
        o = -(-num // s) + 1
        if (o - 1) * s >= H + p:  # last window must start inside the input (+left pad)
            o -= 1
    else:
        o = num // s + 1
    return o


def _dense(x):
    """Pool kernels need dense channels (ld == C)."""
    if ld_of(x) != x.shape[1]:
        return x.contiguous(memory_format=CL)
    return x


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p, ceil_mode, join=None, stats_box=None):
        N, C, H, W = x.shape
        P = pool_out(H, k[0], s[0], p[0], ceil_mode)
        Q = pool_out(W, k[1], s[1], p[1], ceil_mode)
        y = torch.empty((N, C, P, Q), dtype=BF16, device=x.device, memory_format=CL)
        idx = torch.empty((N, P, Q, C), dtype=torch.uint8, device=x.device) if x.requires_grad else None
        rc = lib().maxpool_fwd(ptr(x), ptr(y), ptr(idx), N, H, W, C, P, Q, k[0], k[1], s[0], s[1], p[0], p[1],
                               stream_handle(), stats=ptr(stats_box[0]) if stats_box else 0)
        if stats_box:
            stats_box[1] = rc == 0
        ctx.save_for_backward(idx)
        ctx.cfg = (x.shape, k, s, p, P, Q)
        ctx.join = join
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        shape, k, s, p, P, Q = ctx.cfg
        N, C, H, W = shape
        dy = _dense(grad_nhwc(dy))
        dx = torch.empty((N, C, H, W), dtype=BF16, device=dy.device, memory_format=CL)
        lib().maxpool_bwd(ptr(dy), ptr(idx), ptr(dx), N, H, W, C, P, Q, k[0], k[1], s[0], s[1], p[0], p[1], stream_handle())
        if ctx.join is not None:
            dx = ctx.join.produce(dx)
        return dx, None, None, None, None, None, None


def max_pool2d(x, kernel_size, stride=None, padding=0, ceil_mode=False, input_join=None, stats_buf=None):
    """``input_join`` (conv.GradJoin): x's gradient is stashed there for another consumer of x to
    sum in its own backward pass (an hourglass level input, models/hourglass.py) -- only when x
    is used as is (no layout copy in between). ``stats_buf``: as upsample_add (returns (y, stats
    or None))."""
    k = _pair(kernel_size)
    s = _pair(stride if stride is not None else kernel_size)
    p = _pair(padding)
    box = [stats_buf, False] if stats_buf is not None else None
    if not native(x):
        y = TF.max_pool2d(x, k, s, p, ceil_mode=ceil_mode)
        return (y, None) if box is not None else y
    xd = _dense(as_nhwc(x, pad_to8=False))
    y = _MaxPoolFn.apply(xd, k, s, p, ceil_mode, input_join if xd is x else None, box)
    return (y, stats_buf if box[1] else None) if box is not None else y


class _AvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p, ceil_mode, cip, divover):
        N, C, H, W = x.shape
        P = pool_out(H, k[0], s[0], p[0], ceil_mode)
        Q = pool_out(W, k[1], s[1], p[1], ceil_mode)
        y = torch.empty((N, C, P, Q), dtype=BF16, device=x.device, memory_format=CL)
        lib().avgpool_fwd(ptr(x), ptr(y), N, H, W, C, P, Q, k[0], k[1], s[0], s[1], p[0], p[1], int(cip), int(divover),
                          stream_handle())
        ctx.cfg = (x.shape, k, s, p, P, Q, cip, divover)
        return y

    @staticmethod
    def backward(ctx, dy):
        shape, k, s, p, P, Q, cip, divover = ctx.cfg
        N, C, H, W = shape
        dy = _dense(grad_nhwc(dy))
        dx = torch.empty((N, C, H, W), dtype=BF16, device=dy.device, memory_format=CL)
        lib().avgpool_bwd(ptr(dy), ptr(dx), N, H, W, C, P, Q, k[0], k[1], s[0], s[1], p[0], p[1], int(cip), int(divover),
                          stream_handle())
        return dx, None, None, None, None, None, None


def avg_pool2d(x, kernel_size, stride=None, padding=0, ceil_mode=False, count_include_pad=True, divisor_override=None):
    k = _pair(kernel_size)
    s = _pair(stride if stride is not None else kernel_size)
    p = _pair(padding)
    if not native(x):
        return TF.avg_pool2d(x, k, s, p, ceil_mode, count_include_pad, divisor_override)
    x = _dense(as_nhwc(x, pad_to8=False))
    return _AvgPoolFn.apply(x, k, s, p, ceil_mode, count_include_pad, divisor_override or 0)


class _GAPFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        N, C, H, W = x.shape
        y = torch.empty((N, C, 1, 1), dtype=BF16, device=x.device, memory_format=CL)
        lib().gap_fwd(ptr(x), ptr(y), N, H * W, C, stream_handle())
        ctx.cfg = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        N, C, H, W = ctx.cfg
        dy = dy.to(BF16).contiguous(memory_format=CL) if not (dy.dtype == BF16 and dy.is_contiguous(memory_format=CL)) else dy
        dx = torch.empty((N, C, H, W), dtype=BF16, device=dy.device, memory_format=CL)
        lib().gap_bwd(ptr(dy), ptr(dx), N, H * W, C, stream_handle())
        return dx


def adaptive_avg_pool2d(x, output_size):
    os_ = _pair(output_size)
    if not native(x) or os_ != (1, 1):
        if native(x):  # general adaptive pooling: exact via avg_pool when divisible
            N, C, H, W = x.shape
            if H % os_[0] == 0 and W % os_[1] == 0:
                kh, kw = H // os_[0], W // os_[1]
                return avg_pool2d(x, (kh, kw), (kh, kw))
            unsupported(f"adaptive_avg_pool2d {H}x{W} -> {os_} (non-divisible)")
        return TF.adaptive_avg_pool2d(x, os_)
    x = _dense(as_nhwc(x, pad_to8=False))
    return _GAPFn.apply(x)


class _UpsampleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, f):
        N, C, H, W = x.shape
        y = torch.empty((N, C, H * f, W * f), dtype=BF16, device=x.device, memory_format=CL)
        lib().upsample_fwd(ptr(x), ptr(y), N, H, W, C, f, stream_handle())
        ctx.cfg = (x.shape, f)
        return y

    @staticmethod
    def backward(ctx, dy):
        (N, C, H, W), f = ctx.cfg
        dy = _dense(grad_nhwc(dy))
        dx = torch.empty((N, C, H, W), dtype=BF16, device=dy.device, memory_format=CL)
        lib().upsample_bwd(ptr(dy), ptr(dx), N, H, W, C, f, stream_handle())
        return dx, None


class _UpsampleAddFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, r, f, stats_box=None):
        N, C, H, W = x.shape
        y = torch.empty_like(r)
        rc = lib().upsample_add(ptr(x), ptr(r), ptr(y), N, H, W, C, f, stream_handle(),
                                stats=ptr(stats_box[0]) if stats_box else 0)
        if stats_box:
            stats_box[1] = rc == 0
        ctx.cfg = (x.shape, f)
        return y

    @staticmethod
    def backward(ctx, dy):
        (N, C, H, W), f = ctx.cfg
        dy = _dense(grad_nhwc(dy))
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty((N, C, H, W), dtype=BF16, device=dy.device, memory_format=CL)
            lib().upsample_bwd(ptr(dy), ptr(dx), N, H, W, C, f, stream_handle())
        return dx, dy, None, None


def upsample_add(x, r, scale_factor=2, stats_buf=None):
    """upsample_nearest(x, scale_factor) + r in one native pass (the Hourglass level merge,
    R/Hourglass/tensorflow/hourglass104.py:95-97); r's gradient is the incoming one unchanged.
    ``stats_buf`` (a BN's [STAT_ROWS, C] statistics workspace): the pass also accumulates the
    batch statistics of its output for the BN that consumes it; returns (y, statistics or None)."""
    f = int(scale_factor)
    box = [stats_buf, False] if stats_buf is not None else None

    def ret(y):
        return (y, stats_buf if box[1] else None) if box is not None else y

    if not native(x) or f != scale_factor:
        from .act import add

        return ret(add(upsample_nearest(x, scale_factor), r))
    x = _dense(as_nhwc(x, pad_to8=False))
    r = _dense(as_nhwc(r, pad_to8=False))
    N, C, H, W = x.shape
    if tuple(r.shape) != (N, C, H * f, W * f) or r.dtype != BF16 or x.dtype != BF16:
        from .act import add

        return ret(add(upsample_nearest(x, scale_factor), r))
    return ret(_UpsampleAddFn.apply(x, r, f, box))


def upsample_nearest(x, scale_factor=2):
    f = int(scale_factor)
    if native(x) and f != scale_factor:
        unsupported(f"nearest upsampling by a non-integer factor {scale_factor}")
    if not native(x):
        return TF.interpolate(x, scale_factor=scale_factor, mode="nearest")
    x = _dense(as_nhwc(x, pad_to8=False))
    return _UpsampleFn.apply(x, f)
