"""Deferred BatchNorm applies: the elementwise BN pass folded into the operand load of the 1x1
conv that consumes its result (csrc/conv_fwd_core.h ``AT_*`` A-operand transforms).

A training BatchNorm cannot be applied in its producer's epilogue (the batch statistics are
complete only when the producer has finished), so the unfused graph spends one full read + write
pass per BN apply, forward and backward. When the consumer is a 1x1 / stride-1 / unpadded conv
(or the dgrad of a 1x1 conv, whose A operand is the incoming gradient row for row), the consumer
can compute the BN output itself while staging its A tile, and the blocks of its first output
column tile store it once as a side output (the materialised tensor the rest of the graph --
wgrad, the next residual join -- still reads). That removes the separate pass's re-read.

Forward (``PendingApply.forward``): ``out = act(x*scale + shift [+ residual | + bn_r(residual)])``
  -- ResNet bottleneck bn2 -> conv3 (AT_BN) and the block's output join -> next block's conv1
  (AT_JOIN, with the activation mask bits the backward needs).
Backward (``PendingApply.backward``): ``dx = kA*dz + kB*x + kC`` -- a BN's input gradient
  consumed by its producing 1x1 conv's dgrad: bn3 -> conv3 dgrad (AT_BWDB, stored mask bits),
  bn1 -> conv1 dgrad (AT_BWDX, mask recomputed from x).

Hand-off rules (every path is safe without the fusion):
  * forward: the BN op returns ``out`` uninitialised with ``out._dv_pending`` set; a consumer
    that can fuse passes it to the kernel, any other native consumer calls ``resolve(out)``
    first, which launches the ordinary apply pass. Only model code that knows its consumer
    asks for a deferred output (models/resnet.py), and the stage's last block never does;
  * backward: the BN backward returns ``dx`` uninitialised and registers it here by storage;
    the producing conv's backward ``take_grad``s it before reading ``dy`` and either fuses it
    into its dgrad or materialises it. A BN only defers when its input is the output of a
    1x1 conv created in the same fused op (ops.bn.conv_bn_act), so that conv's backward is the
    tensor's only consumer.

OFF BY DEFAULT (``DV_DEFER=1`` / ``ENABLED = True`` turns it on): measured on ResNet-50 at batch
256 it loses (profiles/defer_experiment.txt). The separate apply passes already stream at
5-6 TB/s, the best case saves only the consumer's re-read (13 vs 17 tensor-widths of traffic on a
stage-1 join), and both kernel forms tried cost more than that: staging A through registers
breaks the LDS-DMA pipeline (latency-bound K loop), and a per-fragment transform on top of the
DMA pipeline repeats the transform in every output-column tile and wave column and widens the
stages to one block per CU. The kernels are exact (bitwise equal to the unfused step,
tests/test_defer_gpu.py) and stay available for A/B runs.
"""
from __future__ import annotations

import os

import torch

from .common import F32, lib, ptr, stream_handle

AT_BN, AT_JOIN, AT_BWDB, AT_BWDX = 1, 2, 3, 4
ENABLED = os.environ.get("DV_DEFER", "0") not in ("0", "off", "")
COUNTERS = {"fwd_fused": 0, "fwd_materialized": 0, "bwd_fused": 0, "bwd_materialized": 0}

_ONES = {}


def _ones_zeros(C, device):
    key = (str(device), C)
    t = _ONES.get(key)
    if t is None:
        t = _ONES[key] = torch.stack([torch.ones(C, dtype=F32, device=device), torch.zeros(C, dtype=F32, device=device)])
    return t


class PendingApply:
    """A BN elementwise pass not yet run. ``kernel_args()`` are the conv_fwd ``at_*`` arguments
    that fold it into a consumer; ``materialize()`` runs it as the ordinary pass instead."""

    __slots__ = ("at", "out", "x", "r", "bits", "coefs", "act", "slope", "run", "done", "keep")

    def __init__(self, at, out, x, r, bits, coefs, act, slope, run, keep=()):
        self.at, self.out, self.x, self.r, self.bits = at, out, x, r, bits
        self.coefs, self.act, self.slope, self.run = coefs, act, slope, run
        self.keep = keep  # tensors the coefficient views point into
        self.done = False

    @classmethod
    def forward(cls, out, x, residual, scale, shift, rscale, rshift, act, slope, bits, run):
        """act(x*scale + shift (+ residual*rscale + rshift | + residual)) into ``out`` (+ mask bits)."""
        if residual is None:
            return cls(AT_BN, out, x, None, bits, (scale, shift), act, slope, run)
        if rscale is None:  # identity residual: the kernel's z = fma(r, 1, z) == z + r exactly
            oz = _ones_zeros(x.shape[1], x.device)
            return cls(AT_JOIN, out, x, residual, bits, (scale, shift, oz[0], oz[1]), act, slope, run, keep=(oz,))
        return cls(AT_JOIN, out, x, residual, bits, (scale, shift, rscale, rshift), act, slope, run)

    @classmethod
    def backward(cls, dx, dout, x, bits, kA, kB, kC, mscale, mshift, act, slope, run):
        """dx = kA*dz + kB*x + kC, dz = act'(.)*dout from ``bits`` or from z = x*mscale + mshift."""
        if bits is not None:
            return cls(AT_BWDB, dx, x, dout, bits, (kA, kB, kC), act, slope, run)
        if not act:
            mscale, mshift = kA, kB  # unused by the kernel (act 0: dz = dout); any aligned vectors
        return cls(AT_BWDX, dx, x, dout, None, (kA, kB, kC, mscale, mshift), act, slope, run)

    def kernel_args(self):
        a = dict(at=self.at, at_act=int(self.act), at_slope=float(self.slope), at_x=ptr(self.x), at_side=ptr(self.out))
        if self.r is not None:
            a["at_r"] = ptr(self.r)
        if self.bits is not None:
            a["at_bits_in" if self.at >= AT_BWDB else "at_bits_out"] = ptr(self.bits)
        for j, c in enumerate(self.coefs):
            a[f"at_c{j}"] = ptr(c)
        return a

    def fused(self):
        self.done = True
        COUNTERS["bwd_fused" if self.at >= AT_BWDB else "fwd_fused"] += 1

    def materialize(self):
        if not self.done:
            self.run()
            self.done = True
            COUNTERS["bwd_materialized" if self.at >= AT_BWDB else "fwd_materialized"] += 1
        return self.out


def pending(t):
    """The forward PendingApply of ``t`` that has not run yet, or None."""
    p = getattr(t, "_dv_pending", None) if isinstance(t, torch.Tensor) else None
    return p if (p is not None and not p.done) else None


def resolve(t):
    """Make sure ``t`` holds its values (runs a deferred apply). Returns ``t``."""
    p = pending(t)
    if p is not None:
        p.materialize()
    return t


def fusable_1x1(C, ld, R, S, stride, padding, dilation, groups):
    """Whether a conv's A operand (its input, or the dY of its dgrad) is one dense source row per
    GEMM row with whole 64-channel K-tiles: the AT kernels' geometry (csrc/conv_fwd.hip)."""
    return (R == 1 and S == 1 and tuple(padding) == (0, 0) and tuple(dilation) == (1, 1) and groups == 1
            and C % 64 == 0 and ld == C and C * 5 * 4 + 65536 <= 160 * 1024)


# ---- backward hand-off: BN backward -> its producing conv's backward (by storage) ----
_GRADS = {}


def register_grad(dx, pend):
    _GRADS[dx.data_ptr()] = (pend, tuple(dx.shape), dx.stride())


def take_grad(dy):
    """The pending backward apply whose output buffer is ``dy``, or None."""
    if not _GRADS or not isinstance(dy, torch.Tensor):
        return None
    e = _GRADS.pop(dy.data_ptr(), None)
    if e is None:
        return None
    pend, shape, stride = e
    if pend.done:
        return None
    if tuple(dy.shape) != shape or dy.stride() != stride:  # a different view of the storage: be safe
        pend.materialize()
        return None
    return pend


def flush():
    """Materialise every registered backward apply (an exception path / end of backward)."""
    while _GRADS:
        _, (pend, _, _) = _GRADS.popitem()
        pend.materialize()


def launch_bn_apply(x, residual, out, C, scale, shift, act, slope, mask, rscale=None, rshift=None, post=False):
    lib().bn_apply(ptr(x), ptr(residual), ptr(out), x.numel(), C, ptr(scale), ptr(shift), act, float(slope), ptr(mask),
                   stream_handle(), rscale=ptr(rscale) if rscale is not None else 0,
                   rshift=ptr(rshift) if rshift is not None else 0, post=int(post))
