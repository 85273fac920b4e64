"""Channel concatenation and channel shuffle on native NHWC tensors.

* ``slice_cat(parts)``: the parts were WRITTEN into channel slices of one NHWC buffer by their
  producing kernels (``conv2d(..., out=concat_slices(...)[i])``: the conv epilogue stores at a
  pixel stride of the concat width) -- the concat itself moves no bytes. Inception V1's
  4-branch module (R/Inception/pytorch/models/inception_v1.py:156-158) uses this.
* ``concat(tensors)``: one output buffer, each input copied into its channel slice by a
  16-B-vector native kernel (YOLO routes R/YOLO/tensorflow/yolov3.py:152,181, ShuffleNet's
  stride-2 shortcut, Inception V3 extension).
* ``channel_shuffle(x, groups)``: ShuffleNet's (g, c) -> (c, g) channel transpose as a native
  channel gather; backward gathers with the inverse permutation.

Backward of both concats hands each part the matching channel slice of the incoming gradient
(a strided view: pixel stride = concat width); the conv / BN backward kernels read such views
directly.
"""
from __future__ import annotations

from typing import List, Sequence

import torch

from .common import BF16, CL, alloc_cl, is_nhwc, ld_of, lib, native, ptr, stream_handle


def concat_slices(N: int, channels: Sequence[int], H: int, W: int, device) -> List[torch.Tensor]:
    """Allocate one NHWC buffer for ``sum(channels)`` and return its channel-slice views (the
    producers' output buffers); feed the produced parts to ``slice_cat``."""
    if any(c % 8 for c in channels):
        raise ValueError("write-into-slice concat needs channel counts that are multiples of 8")
    buf = alloc_cl((N, sum(channels), H, W), device=device)
    out, c0 = [], 0
    for c in channels:
        out.append(buf[:, c0:c0 + c])
        c0 += c
    return out


class _SliceCat(torch.autograd.Function):
    @staticmethod
    def forward(ctx, *parts):
        base = parts[0]._base
        ctx.sizes = [p.shape[1] for p in parts]
        return base.as_strided(base.shape, base.stride(), base.storage_offset())

    @staticmethod
    def backward(ctx, g):
        out, c0 = [], 0
        for c in ctx.sizes:
            out.append(g[:, c0:c0 + c])
            c0 += c
        return tuple(out)


def slice_cat(parts: Sequence[torch.Tensor]) -> torch.Tensor:
    """Concatenation of parts that already live, in order, in the channel slices of one buffer."""
    base = parts[0]._base
    c0 = 0
    for p in parts:
        if p._base is not base or p.data_ptr() != base.data_ptr() + c0 * base.element_size():
            raise ValueError("slice_cat parts must be consecutive channel slices of one buffer")
        c0 += p.shape[1]
    if c0 != base.shape[1]:
        raise ValueError("slice_cat parts do not cover the buffer")
    return _SliceCat.apply(*parts)


def _copy_into(src: torch.Tensor, dst: torch.Tensor):
    N, C, H, W = src.shape
    lib().nhwc_copy(ptr(src), ld_of(src), ptr(dst), ld_of(dst), N * H * W, C, 0, stream_handle())


class _Concat(torch.autograd.Function):
    @staticmethod
    def forward(ctx, *xs):
        N, _, H, W = xs[0].shape
        sizes = [x.shape[1] for x in xs]
        out = alloc_cl((N, sum(sizes), H, W), device=xs[0].device)
        c0 = 0
        for x in xs:
            _copy_into(x, out[:, c0:c0 + x.shape[1]])
            c0 += x.shape[1]
        ctx.sizes = sizes
        return out

    @staticmethod
    def backward(ctx, g):
        out, c0 = [], 0
        for c in ctx.sizes:
            out.append(g[:, c0:c0 + c])
            c0 += c
        return tuple(out)


def _vec_ok(t: torch.Tensor) -> bool:
    return is_nhwc(t) and t.shape[1] % 8 == 0 and ld_of(t) % 8 == 0 and t.data_ptr() % 16 == 0


def concat(tensors: Sequence[torch.Tensor]) -> torch.Tensor:
    """torch.cat(tensors, 1) for 4-D activations: native slice copies on the GPU path."""
    if not native(tensors[0]):
        return torch.cat(list(tensors), 1)
    xs = []
    for t in tensors:
        if not _vec_ok(t):
            t = t.to(BF16).contiguous(memory_format=CL)
            if not _vec_ok(t):
                raise NotImplementedError("native concat needs channel counts that are multiples of 8")
        xs.append(t)
    return _Concat.apply(*xs)


_PERM = {}


def _perm(C: int, groups: int, device, inverse: bool) -> torch.Tensor:
    key = (C, groups, str(device), inverse)
    t = _PERM.get(key)
    if t is None:
        c = torch.arange(C).view(groups, C // groups).t().reshape(-1)  # out[j] = in[c[j]]
        if inverse:
            inv = torch.empty_like(c)
            inv[c] = torch.arange(C)
            c = inv
        t = c.to(torch.int32).to(device)
        _PERM[key] = t
    return t


def _gather(x: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    N, C, H, W = x.shape
    y = alloc_cl((N, C, H, W), device=x.device)
    lib().nhwc_copy(ptr(x), ld_of(x), ptr(y), ld_of(y), N * H * W, C, ptr(idx), stream_handle())
    return y


class _Shuffle(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, groups):
        ctx.groups = groups
        return _gather(x, _perm(x.shape[1], groups, x.device, False))

    @staticmethod
    def backward(ctx, g):
        if not is_nhwc(g):
            g = g.to(BF16).contiguous(memory_format=CL)
        return _gather(g, _perm(g.shape[1], ctx.groups, g.device, True)), None


def channel_shuffle(x: torch.Tensor, groups: int) -> torch.Tensor:
    """(N, g*c, H, W) -> channel j*g + i takes input channel i*c + j (ShuffleNet V1)."""
    N, C, H, W = x.shape
    if not native(x):
        return x.reshape(N, groups, C // groups, H, W).transpose(1, 2).reshape(N, C, H, W)
    if not is_nhwc(x):
        x = x.to(BF16).contiguous(memory_format=CL)
    return _Shuffle.apply(x, groups)
