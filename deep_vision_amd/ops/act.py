"""Elementwise activations, residual add, dropout on native bf16 kernels (csrc/elementwise.hip).

Gradients are computed from the activation OUTPUT, so in-place-style memory behaviour of the
reference (``nn.ReLU(inplace=True)``, R/ResNet/pytorch/models/resnet50.py:31) costs nothing
extra: only the output is saved.
"""
from __future__ import annotations

import torch
import torch.nn.functional as TF

from .common import ACT_IDS, BF16, CL, lib, native, ptr, stream_handle


def _native_layout(x):
    """Any bf16 tensor that is dense in *some* memory order can be processed flat."""
    return x.dtype == BF16 and (x.is_contiguous() or x.is_contiguous(memory_format=CL))


def _prep(x):
    if _native_layout(x):
        return x
    if x.dim() == 4:
        return x.to(dtype=BF16).contiguous(memory_format=CL)  # .to() keeps non-dense CL-strided views
    return x.to(dtype=BF16).contiguous()


class _ActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, act, slope):
        y = torch.empty_like(x)
        lib().act_fwd(ptr(x), ptr(y), x.numel(), act, float(slope), stream_handle())
        ctx.save_for_backward(y)
        ctx.cfg = (act, slope)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        act, slope = ctx.cfg
        dy = dy.to(BF16)
        if dy.stride() != y.stride():
            dy = dy.contiguous(memory_format=CL) if y.dim() == 4 and y.is_contiguous(memory_format=CL) else dy.contiguous()
            if dy.stride() != y.stride():
                dy = torch.empty_like(y).copy_(dy)
        dx = torch.empty_like(y)
        lib().act_bwd(ptr(dy), ptr(y), ptr(dx), y.numel(), act, float(slope), stream_handle())
        return dx, None, None


def activation(x, act, slope=0.0):
    if act is None or act == "none":
        return x
    if not native(x):
        if act == "relu":
            return TF.relu(x)
        if act in ("leaky", "leaky_relu"):
            return TF.leaky_relu(x, slope)
        if act == "tanh":
            return torch.tanh(x)
        if act == "sigmoid":
            return torch.sigmoid(x)
        raise ValueError(act)
    return _ActFn.apply(_prep(x), ACT_IDS[act], float(slope))


def relu(x):
    return activation(x, "relu")


def leaky_relu(x, slope=0.01):
    return activation(x, "leaky", slope)


class _AddFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, act, slope):
        y = torch.empty_like(a)
        lib().add(ptr(a), ptr(b), ptr(y), a.numel(), 1.0, 1.0, act, float(slope), stream_handle())
        ctx.save_for_backward(y if act else None)
        ctx.cfg = (act, slope)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        act, slope = ctx.cfg
        dy = dy.to(BF16)
        if act:
            if dy.stride() != y.stride():
                dy = torch.empty_like(y).copy_(dy)
            g = torch.empty_like(y)
            lib().act_bwd(ptr(dy), ptr(y), ptr(g), y.numel(), act, float(slope), stream_handle())
            dy = g
        return dy, dy, None, None


def add(a, b, act=None, slope=0.0):
    """act(a + b) (residual connection)."""
    if not native(a):
        return activation(a + b, act, slope)
    a = _prep(a)
    b = _prep(b)
    if b.stride() != a.stride():
        b = torch.empty_like(a).copy_(b)
    return _AddFn.apply(a, b, ACT_IDS[act], float(slope))


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed, step):
        y = torch.empty_like(x)
        lib().dropout(ptr(x), ptr(y), x.numel(), float(p), seed, stream_handle(), step=ptr(step))
        ctx.cfg = (p, seed, x.stride())
        ctx.step = step
        return y

    @staticmethod
    def backward(ctx, dy):
        p, seed, stride = ctx.cfg
        dy = _prep(dy)
        if dy.stride() != stride:  # the mask is indexed by flat position: match the forward layout
            dy = torch.empty_strided(dy.shape, stride, dtype=dy.dtype, device=dy.device).copy_(dy)
        dx = torch.empty_like(dy)
        lib().dropout(ptr(dy), ptr(dx), dy.numel(), float(p), seed, stream_handle(), step=ptr(ctx.step))  # same mask
        return dx, None, None, None


# Per-device step counters of captured steps: a HIP graph bakes the host seed of every dropout call
# into its launch, so inside a capture the kernels also read this counter, which the replayer
# advances before every replay (train/graph.py CapturedStep) -- fresh masks per replayed step.
_STEP = {}


def step_counter(device):
    dev = torch.device(device) if not isinstance(device, int) else torch.device("cuda", device)
    if dev.type == "cuda" and dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    t = _STEP.get(dev)
    if t is None:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("dropout step counter created inside a capture (CapturedStep makes it first)")
        t = _STEP[dev] = torch.zeros(1, dtype=torch.int32, device=dev)
    return t


def advance_dropout_step():
    """Advance every device's dropout step counter (one tiny kernel each): called per replay."""
    for t in _STEP.values():
        t.add_(1)


def dropout(x, p=0.5, training=True):
    if not training or p == 0.0:
        return x
    if not native(x):
        return TF.dropout(x, p, training)
    x = _prep(x)
    # the host seed comes from torch's global CPU generator: torch.manual_seed makes masks
    # reproducible (deterministic mode)
    seed = int(torch.randint(0, 2**62, (1,)).item())
    step = step_counter(x.device) if torch.cuda.is_current_stream_capturing() else None
    return _DropoutFn.apply(x, p, seed, step)
