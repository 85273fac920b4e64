"""Local response normalisation on the native kernel (csrc/lrn.hip).

``local_response_norm`` follows torch.nn.LocalResponseNorm (used by the reference with
size == channel count, R/AlexNet/pytorch/models/alexnet_v1.py:41, R/Inception/pytorch/models/
inception_v1.py:30,38); ``tf_local_response_norm`` follows tf.nn.local_response_normalization
(R/AlexNet/tensorflow/models/alexnet_v2.py:9-22: depth_radius 5, bias 1, alpha 1, beta 0.5).
"""
from __future__ import annotations

import torch
import torch.nn.functional as TF

from .common import BF16, CL, ld_of, lib, native, ptr, stream_handle


class _LRNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, lo, hi, alpha_eff, beta, k):
        N, C, H, W = x.shape
        y = torch.empty_like(x)
        lib().lrn_fwd(ptr(x), ptr(y), N * H * W, C, lo, hi, float(alpha_eff), float(beta), float(k), stream_handle())
        ctx.save_for_backward(x)
        ctx.cfg = (lo, hi, alpha_eff, beta, k)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        lo, hi, a, b, k = ctx.cfg
        N, C, H, W = x.shape
        dy = dy.to(BF16).contiguous(memory_format=CL)
        dx = torch.empty_like(x)
        lib().lrn_bwd(ptr(x), ptr(dy), ptr(dx), N * H * W, C, lo, hi, float(a), float(b), float(k), stream_handle())
        return dx, None, None, None, None, None


def _dense_nhwc(x):
    x = x.to(BF16)
    if not x.is_contiguous(memory_format=CL) or ld_of(x) != x.shape[1]:
        x = x.contiguous(memory_format=CL)
    return x


def local_response_norm(x, size, alpha=1e-4, beta=0.75, k=1.0):
    if not native(x):
        return TF.local_response_norm(x, size, alpha, beta, k)
    return _LRNFn.apply(_dense_nhwc(x), size // 2, (size - 1) // 2, alpha / size, beta, k)


def tf_local_response_norm(x, depth_radius=5, bias=1.0, alpha=1.0, beta=0.5):
    if not native(x):
        sq = x.pow(2)
        C = x.shape[1]
        s = TF.pad(sq, (0, 0, 0, 0, depth_radius, depth_radius))
        win = sum(s[:, i:i + C] for i in range(2 * depth_radius + 1))
        return x / (bias + alpha * win).pow(beta)
    return _LRNFn.apply(_dense_nhwc(x), depth_radius, depth_radius, alpha, beta, bias)
