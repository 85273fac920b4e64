"""Layer modules: drop-in subclasses of the torch.nn layers used by the reference.

Parameter / buffer names and shapes are exactly torch's, so checkpoints are key-compatible
with the reference's ``state_dict``s (e.g. ``conv2x.0.projection.1.running_mean``). On GPU
tensors ``forward`` dispatches to the native gfx950 kernels (deep_vision_amd.ops).
"""
from __future__ import annotations

import math

import torch
import torch.nn as tnn

from .. import ops as F
from ..ops.common import native, unsupported

__all__ = [
    "Conv2d", "ConvTranspose2d", "Linear", "BatchNorm2d", "ReLU", "LeakyReLU", "Tanh", "Sigmoid", "MaxPool2d",
    "AvgPool2d", "AdaptiveAvgPool2d", "Dropout", "Upsample", "LocalResponseNorm", "Flatten", "Sequential",
    "ZeroPad2d", "ReflectionPad2d", "ChannelShuffle", "Identity", "FusedSequential",
]

Sequential = tnn.Sequential
Flatten = tnn.Flatten
Identity = tnn.Identity


class Conv2d(tnn.Conv2d):
    """torch.nn.Conv2d; ``padding='same_keras'`` reproduces TF/Keras asymmetric 'same' padding
    (extra row/col at the bottom/right at stride 2)."""

    def __init__(self, *args, padding=0, **kw):
        self.keras_same = padding == "same_keras"
        super().__init__(*args, padding=0 if self.keras_same else padding, **kw)

    def native_padding(self, H, W):
        """Padding for ops.conv2d: ``self.padding``, or the Keras 'same' (top, bottom, left,
        right) pads for an H x W input: total = max((ceil(i/s)-1)*s + (k-1)*d + 1 - i, 0), the
        odd pixel at the bottom/right."""
        if not self.keras_same:
            return self.padding
        out = []
        for i, k, s, d in ((H, self.kernel_size[0], self.stride[0], self.dilation[0]),
                           (W, self.kernel_size[1], self.stride[1], self.dilation[1])):
            o = -(-i // s)
            tot = max((o - 1) * s + (k - 1) * d + 1 - i, 0)
            out += [tot // 2, tot - tot // 2]
        return tuple(out) if out[0] != out[1] or out[2] != out[3] else (out[0], out[2])

    def forward(self, x):
        if self.keras_same:
            return F.conv2d(x, self.weight, self.bias, self.stride, self.native_padding(x.shape[2], x.shape[3]),
                            self.dilation, self.groups)
        if self.padding_mode != "zeros":
            if not native(x):
                return super().forward(x)
            if self.padding_mode != "reflect":
                unsupported(f"Conv2d padding_mode={self.padding_mode!r}")
            return F.conv2d(x, self.weight, self.bias, self.stride, self.padding, self.dilation, self.groups,
                            pad_mode="reflect")
        return F.conv2d(x, self.weight, self.bias, self.stride, self.padding, self.dilation, self.groups)


def pad2d(x, pads, mode="constant"):
    """(left, right, top, bottom) padding in the native layout."""
    y = tnn.functional.pad(x, pads, mode=mode)
    if native(x):
        y = y.contiguous(memory_format=torch.channels_last)
    return y


class ConvTranspose2d(tnn.ConvTranspose2d):
    """torch.nn.ConvTranspose2d; ``padding='same_keras'`` gives Keras Conv2DTranspose 'same'
    semantics (output = input * stride, top/left pad (k - s) // 2 -- e.g. k3/s2 differs from
    torch's padding=1, output_padding=1 by a one-pixel shift)."""

    def __init__(self, *args, padding=0, **kw):
        self.keras_same = padding == "same_keras"
        super().__init__(*args, padding=0 if self.keras_same else padding, **kw)

    def forward(self, x, output_size=None):
        if self.keras_same:
            from ..ops.conv import keras_same_transpose

            pad, out = keras_same_transpose(x.shape[2], x.shape[3], self.kernel_size, self.stride)
            return F.conv_transpose2d(x, self.weight, self.bias, self.stride, pad, 0, self.groups, self.dilation,
                                      output_size=out)
        if not native(x):
            return super().forward(x, output_size)
        op = self.output_padding
        if output_size is not None:  # torch semantics: output_size picks the output_padding
            osz = tuple(output_size)[-2:]
            op = tuple(osz[i] - ((x.shape[2 + i] - 1) * self.stride[i] - 2 * self.padding[i]
                                 + self.dilation[i] * (self.kernel_size[i] - 1) + 1) for i in range(2))
            if any(v < 0 or v >= max(self.stride[i], self.dilation[i]) for i, v in enumerate(op)):
                raise ValueError(f"requested output size {osz} is not reachable")
        return F.conv_transpose2d(x, self.weight, self.bias, self.stride, self.padding, op, self.groups,
                                  self.dilation)


class Linear(tnn.Linear):
    def forward(self, x):
        return F.linear(x, self.weight, self.bias)


class BatchNorm2d(tnn.BatchNorm2d):
    def forward(self, x):
        if not native(x):
            return super().forward(x)
        return F.batch_norm_act(x, self)

    # the native path counts num_batches_tracked on the host and writes it lazily (ops/bn.py
    # _count_batch): a copy or pickle takes the exact count, a reset drops the pending steps
    def __getstate__(self):
        from ..ops.bn import _flush_batch_count

        _flush_batch_count(self)
        return super().__getstate__()

    def reset_running_stats(self):
        self.__dict__["_dv_nbt_pending"] = 0
        super().reset_running_stats()


class ReLU(tnn.ReLU):
    def forward(self, x):
        return F.relu(x) if native(x) else super().forward(x)


class LeakyReLU(tnn.LeakyReLU):
    def forward(self, x):
        return F.leaky_relu(x, self.negative_slope) if native(x) else super().forward(x)


class Tanh(tnn.Tanh):
    def forward(self, x):
        return F.activation(x, "tanh") if native(x) else super().forward(x)


class Sigmoid(tnn.Sigmoid):
    def forward(self, x):
        return F.activation(x, "sigmoid") if native(x) else super().forward(x)


class MaxPool2d(tnn.MaxPool2d):
    def forward(self, x):
        if not native(x):
            return super().forward(x)
        if self.dilation not in (1, (1, 1)) or self.return_indices:
            unsupported("MaxPool2d with dilation / return_indices")
        return F.max_pool2d(x, self.kernel_size, self.stride, self.padding, self.ceil_mode)


class AvgPool2d(tnn.AvgPool2d):
    def forward(self, x):
        if not native(x):
            return super().forward(x)
        return F.avg_pool2d(x, self.kernel_size, self.stride, self.padding, self.ceil_mode, self.count_include_pad,
                            self.divisor_override)


class AdaptiveAvgPool2d(tnn.AdaptiveAvgPool2d):
    def forward(self, x):
        return F.adaptive_avg_pool2d(x, self.output_size) if native(x) else super().forward(x)


class Dropout(tnn.Dropout):
    def forward(self, x):
        return F.dropout(x, self.p, self.training) if native(x) else super().forward(x)


class Upsample(tnn.Upsample):
    def forward(self, x):
        if not native(x):
            return super().forward(x)
        if self.mode != "nearest" or self.scale_factor is None:
            unsupported(f"Upsample mode={self.mode!r} / size=")
        return F.upsample_nearest(x, self.scale_factor)


class LocalResponseNorm(tnn.LocalResponseNorm):
    """torch LRN semantics (window ``size`` across channels; the reference uses size = C,
    R/AlexNet/pytorch/models/alexnet_v1.py:41). Native kernel: deep_vision_amd.ops.lrn."""

    def forward(self, x):
        if not native(x):
            return super().forward(x)
        from ..ops.lrn import local_response_norm

        return local_response_norm(x, self.size, self.alpha, self.beta, self.k)


class ZeroPad2d(tnn.ZeroPad2d):
    def forward(self, x):
        return pad2d(x, self.padding) if native(x) else super().forward(x)


class ReflectionPad2d(tnn.ReflectionPad2d):
    def forward(self, x):
        return pad2d(x, self.padding, mode="reflect") if native(x) else super().forward(x)


class ChannelShuffle(tnn.Module):
    """ShuffleNet channel shuffle: (N, g*c, H, W) -> transpose groups (native channel gather)."""

    def __init__(self, groups):
        super().__init__()
        self.groups = groups

    def forward(self, x):
        return F.channel_shuffle(x, self.groups)


_ACTS = {tnn.ReLU: ("relu", None), tnn.LeakyReLU: ("leaky", "negative_slope")}


def _act_of(m):
    for cls, (name, attr) in _ACTS.items():
        if isinstance(m, cls):
            return name, (getattr(m, attr) if attr else 0.0)
    return None, 0.0


class FusedSequential(tnn.Sequential):
    """torch.nn.Sequential that, on native GPU tensors, fuses producer -> activation chains:

    Conv2d [-> BatchNorm2d] [-> ReLU/LeakyReLU]  -> one conv (+BN statistics epilogue, +apply)
    Linear -> ReLU/LeakyReLU                     -> one GEMM with a fused activation epilogue

    Module indices (and therefore state_dict keys) are exactly those of nn.Sequential.
    """

    def forward(self, x):
        if not native(x):
            return super().forward(x)
        mods = list(self._modules.values())
        i = 0
        while i < len(mods):
            m = mods[i]
            nxt = mods[i + 1] if i + 1 < len(mods) else None
            if isinstance(m, (tnn.ZeroPad2d, tnn.ReflectionPad2d)) and isinstance(nxt, Conv2d) and \
                    nxt.padding_mode == "zeros" and not nxt.keras_same and tuple(nxt.padding) == (0, 0):
                # pad -> pad-0 conv: the pad becomes the conv's (asymmetric) padding / reflect gather
                l, r, t, b = m.padding
                act, slope = _act_of(mods[i + 2]) if i + 2 < len(mods) else (None, 0.0)
                if isinstance(m, tnn.ReflectionPad2d):
                    x = F.conv2d(x, nxt.weight, nxt.bias, nxt.stride, (t, l), nxt.dilation, nxt.groups, act=act,
                                 slope=slope, pad_mode="reflect")
                else:
                    x = F.conv2d(x, nxt.weight, nxt.bias, nxt.stride, (t, b, l, r) if (t, l) != (b, r) else (t, l),
                                 nxt.dilation, nxt.groups, act=act, slope=slope)
                i += 3 if act else 2
                continue
            if isinstance(m, Conv2d) and m.padding_mode == "zeros":
                pad = m.native_padding(x.shape[2], x.shape[3])
                if isinstance(nxt, tnn.BatchNorm2d):
                    act, slope = _act_of(mods[i + 2]) if i + 2 < len(mods) else (None, 0.0)
                    x = F.conv_bn_act(x, m, nxt, act, slope)
                    i += 3 if act else 2
                    continue
                act, slope = _act_of(nxt)
                if act:
                    x = F.conv2d(x, m.weight, m.bias, m.stride, pad, m.dilation, m.groups, act=act, slope=slope)
                    i += 2
                    continue
            if isinstance(m, tnn.Linear):
                act, slope = _act_of(nxt)
                if act:
                    x = F.linear(x, m.weight, m.bias, act=act, slope=slope)
                    i += 2
                    continue
            x = m(x)
            i += 1
        return x
