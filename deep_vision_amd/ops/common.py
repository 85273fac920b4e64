"""Shared helpers for the native op layer.

GPU tensor conventions (all native ops):
  * 4-D activations are ``torch.bfloat16`` with ``torch.channels_last`` strides, i.e.
    physically NHWC; the channel stride (``ld``) may exceed the channel count when the
    channel count is not a multiple of 8 (the tensor is then a view of a padded buffer).
  * 2-D activations (Linear in/out) are bf16 row-major.
  * parameters, BN statistics and optimizer state are fp32.
"""
from __future__ import annotations

import os

import torch

from .._ext import lib, ptr, stream_handle  # noqa: F401

BF16 = torch.bfloat16
F32 = torch.float32
CL = torch.channels_last

_FORCE_TORCH = os.environ.get("DV_BACKEND", "native").lower() == "torch"

ACT_IDS = {None: 0, "none": 0, "relu": 1, "leaky": 2, "leaky_relu": 2, "tanh": 3, "sigmoid": 4}


def set_backend(name: str) -> None:
    """'native' (default: HIP kernels on GPU) or 'torch' (PyTorch/MIOpen reference path)."""
    global _FORCE_TORCH
    _FORCE_TORCH = name.lower() == "torch"


def backend() -> str:
    return "torch" if _FORCE_TORCH else "native"


def native(x: torch.Tensor) -> bool:
    """True when ``x`` should run through the hand-written HIP kernels."""
    return x.is_cuda and not _FORCE_TORCH


def unsupported(what: str):
    """A GPU-path op the native kernels do not implement: raise instead of silently running a
    PyTorch/MIOpen kernel (the torch path exists only as the ``--backend torch`` oracle)."""
    raise NotImplementedError(f"no native gfx950 kernel for {what}; use the torch backend "
                              "(set_backend('torch') / --backend torch) for it")


def round8(c: int) -> int:
    return (c + 7) // 8 * 8


def ld_of(x: torch.Tensor) -> int:
    """Pixel (channel) stride of a channels_last 4-D tensor / row stride of a 2-D tensor."""
    st = x.stride()
    if len(st) == 4:
        sz = x.shape
        return st[3] if sz[3] > 1 else (st[2] if sz[2] > 1 else st[0] // max(1, sz[2] * sz[3]))
    return st[0]


def is_nhwc(x: torch.Tensor) -> bool:
    """bf16, channel stride 1, pixel-major packed layout (ld may be padded)."""
    if x.dtype != BF16 or x.dim() != 4:
        return False
    N, C, H, W = x.shape
    s0, s1, s2, s3 = x.stride()
    if C > 1 and s1 != 1:
        return False
    ld = s3 if W > 1 else (s2 if H > 1 else s0 // max(1, H * W))  # ld_of
    if ld < C or ld % 8 != 0 and ld != C:
        return False
    return (W == 1 or s3 == ld) and (H == 1 or s2 == W * ld) and (N == 1 or s0 == H * W * ld)


def empty_nhwc(N: int, C: int, H: int, W: int, device, zero: bool = False) -> torch.Tensor:
    """bf16 NHWC tensor; channel stride padded to a multiple of 8 (returned as a view)."""
    Cp = round8(C)
    buf = torch.empty((N, Cp, H, W), dtype=BF16, device=device, memory_format=CL)
    if zero or Cp != C:  # pad channels must be finite zeros
        buf.zero_()
    return buf if Cp == C else buf[:, :C]


def alloc_cl(shape, zero=False, device=None, dtype=BF16):
    """channels_last allocation (torch.zeros does not take memory_format)."""
    t = torch.empty(shape, dtype=dtype, device=device, memory_format=CL)
    return t.zero_() if zero else t


def as_nhwc(x: torch.Tensor, pad_to8: bool = True) -> torch.Tensor:
    """Convert any 4-D tensor into the native layout (differentiable when needed)."""
    if is_nhwc(x) and (not pad_to8 or ld_of(x) % 8 == 0):
        return x
    N, C, H, W = x.shape
    if not x.requires_grad and x.dtype in (F32, BF16) and x.is_contiguous() and (pad_to8 or C % 8 == 0):
        Cp = round8(C) if pad_to8 else C
        y = torch.empty((N, Cp, H, W), dtype=BF16, device=x.device, memory_format=CL)
        lib().to_nhwc(ptr(x), int(x.dtype == F32), ptr(y), N, C, H, W, Cp, stream_handle())
        return y  # padded channels are written as zeros by the kernel
    y = x.to(dtype=BF16).contiguous(memory_format=CL)
    if pad_to8 and C % 8 != 0:
        y = torch.nn.functional.pad(y, (0, 0, 0, 0, 0, round8(C) - C)).contiguous(memory_format=CL)
    return y


def grad_nhwc(g: torch.Tensor) -> torch.Tensor:
    """Incoming gradient -> native layout with a channel stride that is a multiple of 8."""
    if is_nhwc(g) and ld_of(g) % 8 == 0:
        return g
    N, C, H, W = g.shape
    out = empty_nhwc(N, C, H, W, g.device, zero=(C % 8 != 0))
    out.copy_(g)
    return out


def like_layout(t: torch.Tensor, ref: torch.Tensor) -> torch.Tensor:
    """``t`` (same logical shape as the NHWC tensor ``ref``) in exactly ``ref``'s physical layout,
    copying when needed. Elementwise kernels that walk two tensors as flat arrays (activation
    backward: dY against the saved Y) need identical strides -- an incoming gradient can be a
    channel slice of a concat (Inception / YOLO route), whose pixel stride is the concat width."""
    if t.dtype == ref.dtype and t.stride() == ref.stride() and t.shape == ref.shape:
        return t
    out = empty_layout(ref)
    out.copy_(t)
    return out


def empty_layout(ref: torch.Tensor) -> torch.Tensor:
    """Uninitialised tensor with ``ref``'s NHWC layout (a dense channels_last tensor, or an
    ``empty_nhwc`` padded view whose whole padded buffer is allocated and zero-padded)."""
    N, C, H, W = ref.shape
    if ld_of(ref) == C:
        return torch.empty_like(ref, memory_format=CL)
    return empty_nhwc(N, C, H, W, ref.device)


def act_grad(dy: torch.Tensor, y: torch.Tensor, act: int, slope: float) -> torch.Tensor:
    """act'(y) * dy for a fused conv activation, as a DENSE NHWC tensor. ``y`` (the saved output)
    and ``dy`` may be channel-slice views of concat buffers (pixel stride > C): the kernel walks
    rows x C with each tensor's own stride, never the flat span of a strided view."""
    N, C, H, W = y.shape
    Cp = round8(C)
    g = empty_nhwc(N, C, H, W, y.device)
    for t in (dy, y):
        if not is_nhwc(t) or ld_of(t) < Cp or ld_of(t) % 8:
            raise ValueError("act_grad: operands must be NHWC with a padded pixel stride >= round8(C)")
    lib().act_bwd_rows(ptr(dy), ld_of(dy), ptr(y), ld_of(y), ptr(g), ld_of(g), N * H * W, Cp, act, float(slope),
                       stream_handle())
    return g


def nhwc_numel(t: torch.Tensor) -> int:
    """Elements spanned by an NHWC tensor including channel padding (flat kernel length)."""
    N, C, H, W = t.shape
    return N * H * W * ld_of(t)


# ---------------------------------------------------------------------------------------------
# Gradient sinks: native backward kernels write parameter gradients straight into the live
# ``param.grad`` buffer (a view into the flat gradient buffer of parallel.flat / train.optim)
# with accumulate semantics — exactly AccumulateGrad's in-place ``grad += g`` without the
# extra pass — and return None to autograd. Readiness for the data-parallel layer is NOT
# signalled here: every use of a parameter still has its autograd edge to the parameter's
# AccumulateGrad node, so the post-accumulate hook (parallel.ddp) fires once, after the LAST
# use's backward (sink or not), which is the only per-step-complete signal.
# ---------------------------------------------------------------------------------------------
def grad_sink(param):
    """The tensor to accumulate ``param``'s gradient into, or None (fall back to autograd).
    Only leaf parameters sink: a non-leaf (e.g. a padded view of a weight) has no live
    ``.grad`` and its gradient must flow back through autograd."""
    if param is None or not param.requires_grad or not param.is_leaf:
        return None
    g = param.grad
    if g is None or g.dtype != F32 or not g.is_contiguous() or g.shape != param.shape or g.device != param.device:
        return None
    if torch.is_grad_enabled():  # double-backward: keep autograd semantics
        return None
    return g


def workspace(owner, key, shape, device, dtype=F32):
    """Persistent zero-initialised buffer owned by a module (self-cleaning accumulators)."""
    ws = owner.__dict__.get("_dv_ws")
    if ws is None:
        ws = owner.__dict__["_dv_ws"] = {}
    if type(device) is not torch.device:
        device = torch.device(device)
    k = (key, shape if type(shape) is tuple else tuple(shape), device, dtype)
    t = ws.get(k)
    if t is None:
        t = torch.zeros(shape, dtype=dtype, device=device)
        ws[k] = t
    return t


def fast_apply(fn_cls):
    """``fn_cls.apply`` without torch's per-call Python wrapper work: autograd.Function.apply runs
    every argument through functorch's dead-wrapper unwrapping (a generator over the ~20-26
    arguments of the conv / BatchNorm Functions, ~3 us per call on the launch-bound models) before
    reaching the C++ apply. Under functorch transforms (never used by the framework) the full path
    is taken."""
    raw = super(torch.autograd.Function, fn_cls).apply
    active = torch._C._are_functorch_transforms_active

    def apply(*args):
        if active():
            return fn_cls.apply(*args)
        return raw(*args)

    return apply

