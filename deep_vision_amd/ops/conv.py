"""Convolution / transposed convolution / linear on the native implicit-GEMM kernels.

Forward   : csrc/igemm.hip MODE_FWD (im2col gather by LDS-DMA, MFMA 16x16x32 bf16)
dgrad     : MODE_FWD on dY with transposed weights: stride 1 via negative pad/dilation,
            1x1-strided via a scattered output map, other strides via the divisibility gather
wgrad     : MODE_WGRAD, split-K over pixels, fp32 accumulate
Epilogue  : bias, ReLU/LeakyReLU, BatchNorm statistics (consumed by ops.bn)

Reference semantics: torch.nn.Conv2d as used by every PT model of the reference, e.g.
R/ResNet/pytorch/models/resnet50.py:20-27 (7x7 s2 stem), :101-133 (bottleneck 1x1/3x3/1x1).
"""
from __future__ import annotations

import contextlib
import os

import torch
import torch.nn.functional as TF

from .. import policy as _policy
from . import wcache
from .common import (ACT_IDS, BF16, CL, F32, act_grad, alloc_cl, as_nhwc, empty_nhwc, fast_apply, grad_nhwc, grad_sink, is_nhwc,
                     ld_of, lib,
                     like_layout, empty_layout, native, nhwc_numel, ptr, round8, stream_handle)

STAT_SHARDS = 64
STAT_ROWS = 2 * STAT_SHARDS + 1  # forward statistics: shard sums + the shift row (csrc/kernels.h)


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


def out_size(H, W, R, S, stride, padding, dilation):
    sh, sw = stride
    ph, pw = padding
    dh, dw = dilation
    P = (H + 2 * ph - dh * (R - 1) - 1) // sh + 1
    Q = (W + 2 * pw - dw * (S - 1) - 1) // sw + 1
    return P, Q


def norm_padding(padding):
    """int | (ph, pw) | (top, bottom, left, right) -> ((pt, pl), (eb, er)).

    The 4-tuple form is TF/Keras asymmetric 'same' padding: the kernels take the top/left pad and
    an output size that includes the ``eb``/``er`` extra bottom/right rows, whose reads fall
    outside the image and are zero-filled by the gather -- no padded copy of the input."""
    if isinstance(padding, int):
        return (padding, padding), (0, 0)
    if len(padding) == 4:
        pt, pb, pl, pr = padding
        if pb < pt or pr < pl:
            raise NotImplementedError("asymmetric padding larger at top/left")
        return (pt, pl), (pb - pt, pr - pl)
    return tuple(padding), (0, 0)


def _prep_weight(weight: torch.Tensor, G: int, pad: int, mode: int, param=None) -> torch.Tensor:
    """fp32 OIHW -> bf16 kernel operand (cached per parameter, see ops/wcache.py).

    mode 0: [G][Og][R][S][pad]  (inner = input channels, zero-padded to ``pad``)
    mode 1: [G][Ig][R][S][pad]  (inner = output channels per group, zero-padded to ``pad``)
    ``param``: the nn.Parameter behind ``weight`` when ``weight`` is a view of it (Linear).
    """
    O, Ig, R, S = weight.shape
    Og = O // G
    n = G * (Og if mode == 0 else Ig) * R * S * pad

    def compute(out):
        w = weight.detach()
        if w.dtype != F32 or not w.is_contiguous():
            w = w.float().contiguous()
        if out is None:
            out = torch.empty(n, dtype=BF16, device=w.device)
        lib().wprep(ptr(w), ptr(out), G, Og, Ig, R, S, pad, mode, 0, stream_handle())
        return out

    key = param if param is not None else weight
    if isinstance(key, torch.nn.Parameter) and key.dtype == F32 and key.is_contiguous():
        return wcache.get(key, G, pad, mode, compute)
    return compute(None)


_CSUM_WS = {}


def _channel_sum(dy: torch.Tensor, out=None) -> torch.Tensor:
    """Per-channel fp32 sum of an NHWC bf16 tensor (bias gradient): csrc/bn.hip dv_channel_sum, two
    launches into a self-cleaning per-device workspace. ``out`` (a gradient sink): added into."""
    N, C, H, W = dy.shape
    ld = ld_of(dy)
    key = (str(dy.device), ld, stream_handle())  # per stream: concurrent branches (models/hourglass.py)
    acc = _CSUM_WS.get(key)
    if acc is None:
        acc = _CSUM_WS[key] = torch.zeros((STAT_ROWS, ld), dtype=F32, device=dy.device)
    dst = out if out is not None else torch.empty(C, dtype=F32, device=dy.device)
    lib().channel_sum(ptr(dy), N * H * W, ld, C, ptr(acc), ptr(dst), int(out is not None), stream_handle())
    return dst


class ColsumBox:
    """Bias-gradient hand-off from a consumer BatchNorm's backward apply pass (ops.bn, csrc/bn.hip
    bn_bwd_apply colsum): the BN of a conv output sums its input gradient per channel while writing
    it, into ``acc`` (self-cleaning shards), and tags the gradient tensor; the producing conv's
    backward folds the shards into its bias gradient when the gradient it receives is exactly that
    tensor (same object, same version -- no other gradient was added to it), instead of a reduction
    pass over it. Otherwise the shards are cleared and the conv reduces dy itself."""

    __slots__ = ("acc", "pending", "version")

    def __init__(self, acc):
        self.acc, self.pending, self.version = acc, False, -1


COUNTERS_BIAS = {"colsum_fused": 0, "colsum_pass": 0}


def _bias_grad(bias, dy, box=None):
    """Bias gradient straight into the live gradient buffer when there is one (None to autograd)."""
    sink = grad_sink(bias)
    if box is not None and box.pending:
        box.pending = False
        if getattr(dy, "_dv_colsum", None) is box and dy._version == box.version:
            COUNTERS_BIAS["colsum_fused"] += 1
            C = dy.shape[1]
            db = sink if sink is not None else torch.empty(C, dtype=F32, device=dy.device)
            lib().channel_sum_finalize(ptr(box.acc), C, C, ptr(db), int(sink is not None), stream_handle())
            return None if sink is not None else db
        box.acc.zero_()
    COUNTERS_BIAS["colsum_pass"] += 1
    db = _channel_sum(dy, out=sink)
    return None if sink is not None else db


def gemm_ksplit(M, N, K):
    """Split-K factor for a GEMM-shaped launch (Linear fwd/dgrad): the 128x128 (or 256x64 for
    N <= 64) tile grid of a short-M GEMM leaves most of the 256 CUs idle -- VGG16's 25088->4096
    at batch 128 is 32 tiles -- so K is split until there are ~256 blocks, keeping >= 512 of K
    per split (csrc/conv_fwd.hip splitk_finalize_kernel sums the fp32 slabs in order)."""
    if N % 4 or K < 1024:
        return 1
    tiles = -(-M // 256) if N <= 64 else -(-M // 128) * -(-N // 128)
    if tiles >= 128:
        return 1
    return max(1, min(16, 256 // tiles, K // 512))


def conv_ksplit(M, O, K, G=1):
    """Split-K factor of a conv whose output grid is too small to fill the chip (Hourglass /
    CenterNet 4x4-16x16 scales: 4-64 tiles): the finalize pass then applies bias, activation,
    residual and the BatchNorm statistics (csrc/conv_fwd.hip splitk_finalize_kernel)."""
    if G != 1 or O % 4 or K < 512:
        return 1
    tiles = -(-M // 256) if O <= 64 else -(-M // 128) * -(-O // 128)
    if tiles >= 64:
        return 1
    return max(1, min(16, 192 // tiles, K // 128))


DGRAD_SPLIT = os.environ.get("DV_DGRAD_SPLIT", "1") != "0"
FIN_BNR = os.environ.get("DV_FIN_BNR", "1") != "0"  # split-K dgrads: BN-backward sums in the finalize pass


def dgrad_ksplit(M, O, K, G=1):
    """Split-K factor of a stride-1 dgrad whose 128x128 tile grid fills less than half of the 256
    CUs and whose K is long (>= 2048): up to 4 splits, >= 1024 of K each (profiles/conv_bench_
    yolov3_vs_miopen.txt: the 13x13 3x3 dgrads)."""
    if not DGRAD_SPLIT or G != 1 or O % 4 or K < 2048:
        return 1
    tiles = -(-M // 128) * -(-O // 128)
    if tiles >= 128:
        return 1
    return max(1, min(4, 256 // tiles, K // 1024))


def conv_fwd_raw(x, wk, y, bias, stats, N, H, W, Cg, ldx, G, Kout, P, Q, R, S, stride, padding, dilation,
                 act=0, slope=0.0, tgather=0, omap=None, ldy=None, res=None, bnref=None, resmask=None, reflect=False,
                 ksplit=1, zfill=0, wlayout=None):
    """Launch the implicit-GEMM kernel. ``bnref`` (ops.bn.BNRef): also reduce that BatchNorm's
    backward statistics over ``y`` in the epilogue; returns True when that was done.
    ``resmask`` (bits, act, slope): ``res`` is a raw gradient masked by act'() before the add."""
    sh, sw = stride
    ph, pw = padding
    dh, dw = dilation
    if stats is not None and stats.numel() < STAT_ROWS * G * Kout:  # the kernel reads the shift row
        raise ValueError(f"conv_fwd_raw: statistics buffer of {stats.numel()} floats < {STAT_ROWS} x {G * Kout}")
    OH, OW, osh, osw, oph, opw = omap if omap is not None else (P, Q, 1, 1, 0, 0)
    bn = {}
    if bnref is not None:
        bn = dict(bnx=ptr(bnref.x), bnbits=ptr(bnref.bits), bnprm=ptr(bnref.prm), bnacc=ptr(bnref.acc),
                  bnmode=bnref.mode, bnact=bnref.act, bnslope=float(bnref.slope))
        if bnref.x2 is not None:  # the folded projection BN of the same residual join (same dz)
            bn.update(bnx2=ptr(bnref.x2), bnprm2=ptr(bnref.prm2), bnacc2=ptr(bnref.acc2))
    if resmask is not None:
        bn.update(resbits=ptr(resmask[0]), resact=int(resmask[1]), resslope=float(resmask[2]))
    if reflect:
        bn["reflect"] = 1
    if zfill:
        bn["zfill"] = 1
    if ksplit > 1:  # fp32 slabs [ksplit][M][Kout], summed + bias + act by the finalize pass
        part = torch.empty((ksplit, N * P * Q, Kout), dtype=F32, device=y.device)
        bn.update(ksplit=int(ksplit), ypart=ptr(part))
    if wlayout is not None:  # (row stride, tap-row stride, tap stride) of a tap subset read in place
        bn.update(w_ld=int(wlayout[0]), w_kr=int(wlayout[1]), w_ks=int(wlayout[2]))
    r = lib().conv_fwd(ptr(x), ptr(wk), ptr(y), ptr(bias), ptr(stats), N, H, W, Cg, ldx, G, Kout, P, Q, R, S, sh, sw,
                       ph, pw, dh, dw, tgather, OH, OW, osh, osw, oph, opw, ldy if ldy is not None else ld_of(y), act,
                       float(slope), ptr(res), stream_handle(), **bn)
    return bnref is not None and r == 0


def _gather_channels(t: torch.Tensor, per_group: int, G: int) -> int:
    """Channels per group the gather kernel reads from ``t`` (must be a multiple of 8).

    For G == 1 a channel count that is not a multiple of 8 is served by reading the zeroed
    padding channels of the buffer (the matching weight rows are zero-padded)."""
    if per_group % 8 == 0:
        return per_group
    if G == 1 and ld_of(t) % 8 == 0:
        return ld_of(t)
    raise NotImplementedError(f"grouped conv with {per_group} channels per group (needs % 8 == 0)")


def _accumulable(t, shape):
    """True when ``t`` can serve as the in-place accumulation target of a dgrad (dense NHWC)."""
    return (t is not None and t.dtype == BF16 and tuple(t.shape) == tuple(shape)
            and t.is_contiguous(memory_format=CL))


def _dgrad(dy, weight, x_shape, Cg_x, G, stride, padding, dilation, device, accum=None, bnref=None):
    """dX (N, G*Cg_x, H, W) from dY; Cg_x may include zero-padding channels.

    ``accum``: a dense gradient of the same input from another consumer (residual shortcut /
    projection); the dgrad kernel adds into it in place (epilogue ``res`` aliasing ``y``),
    replacing autograd's separate gradient-sum pass. A ``MaskedGrad`` accum (a residual block's
    raw output gradient + its ReLU mask bits) is masked inside the same epilogue: the shortcut
    gradient is never materialised."""
    N, _, H, W = x_shape
    O, Ig, R, S = weight.shape
    Og = O // G
    _, _, P, Q = dy.shape
    sh, sw = stride
    ph, pw = padding
    dh, dw = dilation
    Cg_dy = _gather_channels(dy, Og, G)
    wd = _prep_weight(weight, G, Cg_dy, mode=1)  # [G][Ig][R][S][Cg_dy]
    ldy_in = ld_of(dy)
    scatter = (sh, sw) != (1, 1) and R == 1 and S == 1 and (ph, pw) == (0, 0)
    resmask = None
    if isinstance(accum, MaskedGrad):
        if ((sh, sw) == (1, 1) and G == 1 and Cg_x == Ig and _accumulable(accum.grad, (N, G * Cg_x, H, W))):
            resmask = (accum.bits, accum.act, accum.slope)
            accum = accum.grad
        else:
            accum = accum.materialize()
    zfill = 0
    if accum is not None and Cg_x == Ig and _accumulable(accum, (N, G * Cg_x, H, W)):
        dX, res = accum, accum  # scattered positions get res + val, the others keep res
    else:
        # a strided 1x1 scatter zeroes the pixels its taps never reach in the same epilogue
        # (no separate fill pass) when the output is one dense group
        zfill = int(scatter and Cg_x == Ig and G == 1 and Ig % 8 == 0 and H <= P * sh and W <= Q * sw)
        dX, res = alloc_cl((N, G * Cg_x, H, W), zero=((scatter and not zfill) or Cg_x != Ig), device=device), None
    if (sh, sw) == (1, 1):
        # an under-filled grid (small maps, long K: YOLOv3's 13x13 3x3 dgrads, 88 tiles of 128x128 on
        # 256 CUs, K = 9216) splits K across blocks; the BatchNorm-backward sums (modes 1 / 2, one
        # BN) then come from the split-K finalize pass that stores dX (csrc/conv_fwd.hip FinBnr)
        ks = dgrad_ksplit(N * H * W, Ig, R * S * Cg_dy, G) if resmask is None else 1
        fuse = (bnref if (bnref is not None and G == 1 and Cg_x == Ig and (res is not None or accum is None)
                          and (ks == 1 or (FIN_BNR and bnref.mode in (1, 2) and bnref.x2 is None and res is None)))
                else None)
        if conv_fwd_raw(dy, wd, dX, None, None, N, P, Q, Cg_dy, ldy_in, G, Ig, H, W, R, S, (1, 1), (-ph, -pw),
                        (-dh, -dw), ldy=G * Cg_x, res=res, bnref=fuse, resmask=resmask, ksplit=ks):
            fuse.mark_fused(dX)
    elif scatter:
        # the BatchNorm-backward sums ride on the scatter too (the unwritten pixels' zero gradient
        # adds nothing): the stage-transition blocks' shortcut + conv1 dgrads, accumulating last
        fuse = (bnref if (bnref is not None and G == 1 and Cg_x == Ig and not zfill and (res is not None or accum is None))
                else None)
        if conv_fwd_raw(dy, wd, dX, None, None, N, P, Q, Cg_dy, ldy_in, G, Ig, P, Q, 1, 1, (1, 1), (0, 0), (1, 1),
                        omap=(H, W, sh, sw, 0, 0), ldy=G * Cg_x, res=res, zfill=zfill, bnref=fuse):
            fuse.mark_fused(dX)
    elif SUBPIXEL_DGRAD and tuple(dilation) == (1, 1) and Cg_dy % 64 == 0 and R <= 16 and S <= 16:
        _subpixel_dgrad(dy, wd, dX, res, bnref, N, H, W, P, Q, Cg_dy, ldy_in, G, Ig, Cg_x, R, S, stride, padding)
    else:
        COUNTERS_DGRAD["tgather"] += 1
        conv_fwd_raw(dy, wd, dX, None, None, N, P, Q, Cg_dy, ldy_in, G, Ig, H, W, R, S, stride, padding, dilation,
                     tgather=1, ldy=G * Cg_x, res=res)
    if accum is not None and res is None:  # layout mismatch: plain add
        dX = dX[:, : accum.shape[1]] + accum if dX.shape[1] != accum.shape[1] else dX + accum
    return dX


# Strided dgrad (and ConvTranspose forward) by output parity: for stride s every output pixel
# (s*u + a, s*v + b) receives exactly the taps r = a + ph (mod s), s' = b + pw (mod s) -- a dense
# stride-1 sub-convolution of dY with a (ceil(R/s) x ceil(S/s))-ish tap subset, scattered to the
# parity's output grid (omap offset (a, b)). The s*s sub-convolutions cover every output pixel
# once and read the cached full-filter weight in place (strided taps, csrc ConvFwdArgs w_kr/w_ks)
# on the fast LDS-DMA loader; the one-pass transposed gather they replace tests divisibility per
# tap and fetches s*s times the taps it uses (YOLOv3's 3x3/2 downsampling dgrads: 290-380 us).
SUBPIXEL_DGRAD = True
COUNTERS_DGRAD = {"subpixel": 0, "tgather": 0}


def _subpixel_parts(H, W, P, Q, R, S, stride, padding):
    """[(a, b, r0, s0, Ra, Sb, d_h, d_w, U, V)] per output parity: first tap, tap counts, the tap
    offsets' max (as negative padding), sub-output extent; parities no tap reaches have Ra or Sb 0."""
    sh, sw = stride
    ph, pw = padding
    parts = []
    for a in range(min(sh, H)):
        rs = [r for r in range(R) if (r - a - ph) % sh == 0]
        U = -(-(H - a) // sh)
        for b in range(min(sw, W)):
            ss = [t for t in range(S) if (t - b - pw) % sw == 0]
            V = -(-(W - b) // sw)
            dh = (a + ph - rs[0]) // sh if rs else 0
            dw = (b + pw - ss[0]) // sw if ss else 0
            parts.append((a, b, rs[0] if rs else 0, ss[0] if ss else 0, len(rs), len(ss), dh, dw, U, V))
    return parts


# The parity parts write disjoint pixels and each fills a quarter of the grid: launched on streams of
# their own they run side by side (YOLOv3's stride-2 3x3 dgrads; DV_SUBPIXEL_CONC=0: one stream).
# Not in deterministic mode (the parts' BatchNorm-backward partial rows share one slab sequence).
SUBPIXEL_CONC = os.environ.get("DV_SUBPIXEL_CONC", "1") != "0"
_SUBPIX_STREAMS = {}


def _subpix_streams(device, n):
    """n side streams of ``device``, or None inside a capture that would have to create one (a
    captured step's eager warm-up creates them; a capture without one keeps a single stream)."""
    lst = _SUBPIX_STREAMS.setdefault(device, [])
    if len(lst) < n and torch.cuda.is_current_stream_capturing():
        return None
    while len(lst) < n:
        lst.append(torch.cuda.Stream(device=device))
    return lst[:n]


def _subpixel_dgrad(dy, wd, dX, res, bnref, N, H, W, P, Q, Cg_dy, ldy_in, G, Ig, Cg_x, R, S, stride, padding):
    sh, sw = stride
    parts = _subpixel_parts(H, W, P, Q, R, S, stride, padding)
    live = [p for p in parts if p[4] and p[5] and p[8] > 0 and p[9] > 0]
    if len(live) < len(parts) and res is None:
        dX.zero_()  # output parities no tap reaches keep zero gradient
    # the BatchNorm-backward sums ride on every part (disjoint pixels, together all of them), or
    # on none: a partial fusion would leave part of the sums in the accumulator
    fuse = bnref if (bnref is not None and G == 1 and Cg_x == Ig and len(live) == len(parts)) else None
    conc = SUBPIXEL_CONC and dy.is_cuda and len(live) > 1 and not lib().deterministic()
    sides = _subpix_streams(dy.device, len(live) - 1) if conc else None
    conc = sides is not None
    if conc:
        cur = torch.cuda.current_stream(dy.device)
        for st in sides:
            st.wait_stream(cur)
    ok = []
    for idx, (a, b, r0, s0, ra, sb, dh, dw, U, V) in enumerate(live):
        # the parity's taps (r0 + sh*i, s0 + sw*j) of the [G][Ig][R][S][Cg_dy] operand, read in place
        wsub = wd[(r0 * S + s0) * Cg_dy:]
        COUNTERS_DGRAD["subpixel"] += 1
        with (torch.cuda.stream(sides[idx - 1]) if conc and idx > 0 else contextlib.nullcontext()):
            ok.append(conv_fwd_raw(dy, wsub, dX, None, None, N, P, Q, Cg_dy, ldy_in, G, Ig, U, V, ra, sb, (1, 1),
                                   (-dh, -dw), (-1, -1), omap=(H, W, sh, sw, a, b), ldy=G * Cg_x, res=res,
                                   bnref=fuse, wlayout=(R * S * Cg_dy, sh * S * Cg_dy, sw * Cg_dy)))
    if conc:
        for st in sides:
            cur.wait_stream(st)
            for t in (dy, wd, dX):  # the caching allocator must not recycle them under a side stream
                t.record_stream(st)
    if fuse is not None:
        if all(ok):
            fuse.mark_fused(dX)
        elif any(ok):  # mixed acceptance (not expected): drop the partial sums, the BN reduces itself
            fuse.acc.zero_()


class MaskedGrad:
    """A residual block's shortcut gradient in factored form: ``act'(z) * grad`` with the
    activation mask stored as bits by the forward BN+add+ReLU pass (ops.bn). The consumer conv's
    dgrad epilogue applies the mask while adding (csrc/conv_fwd.hip ``resbits``), so the masked
    tensor is never written. ``grad`` is owned by this object and may be overwritten in place."""

    __slots__ = ("grad", "bits", "act", "slope", "coef")

    def __init__(self, grad, bits, act, slope):
        self.grad, self.bits, self.act, self.slope = grad, bits, act, slope

    def materialize(self):
        from .bn import masked_grad

        return masked_grad(self.grad, self.bits, self.act, self.slope)

    def __add__(self, other):
        return self.materialize() + (other.materialize() if isinstance(other, MaskedGrad) else other)

    __radd__ = __add__


def _reflect_dgrad(dy, weight, x, Cg_x, G, stride, padding, dilation):
    """dX of a reflection-padded conv: the dgrad over the padded grid (a pad-0 conv of the padded
    input), then the border folded back onto the pixels it mirrors (csrc reflect_pad_bwd)."""
    N, _, H, W = x.shape
    ph, pw = padding
    dxp = _dgrad(dy, weight, (N, x.shape[1], H + 2 * ph, W + 2 * pw), Cg_x, G, stride, (0, 0), dilation, x.device)
    dx = empty_layout(x) if ld_of(x) == G * Cg_x else alloc_cl((N, G * Cg_x, H, W), device=x.device)
    lib().reflect_pad_bwd(ptr(dxp), ptr(dx), N, H, W, G * Cg_x, ld_of(dxp), ld_of(dx), ph, pw, stream_handle())
    return dx


class GradJoin:
    """Meeting point of two gradients of one tensor (a block input used by a conv and by a
    residual add / projection conv). Whichever backward runs first stashes or announces itself;
    the second folds the sum into the consumer conv's dgrad epilogue (no separate add pass).
    Order-independent: the producer only stashes while the consumer has not run yet.

    Two producers (an hourglass level input: the block's identity shortcut and the pooled low
    branch, models/hourglass.py) fill two slots that a BN backward apply pass sums together
    (take2); a producer on another HIP stream than the consumer (the level's up1 branch runs on a
    side stream) is ordered before it by a stream wait at take time."""

    __slots__ = ("grad", "grad2", "consumer_done", "streams")

    def __init__(self):
        self.grad = self.grad2 = None
        self.consumer_done = False
        self.streams = []

    def produce(self, g):
        """Producer side: returns the gradient to hand to autograd (None when stashed)."""
        if g is None or self.consumer_done:
            return g.materialize() if isinstance(g, MaskedGrad) else g
        t = g.grad if isinstance(g, MaskedGrad) else g
        if t.is_cuda:
            self.streams.append(stream_handle())  # raw handle: no Stream object on the hot path
        if self.grad is None:
            self.grad = g
        elif self.grad2 is None:
            self.grad2 = g
        else:
            self.grad = self.grad + g
        return None

    def can_stash(self):
        """True when a produced gradient would be stashed (not handed to autograd)."""
        return not self.consumer_done and self.grad is None

    def _sync(self, *gs):
        """Order the producers' streams before the current one; the stashed buffers are then in
        use on the current stream too (caching allocator)."""
        if self.streams:
            here = stream_handle()
            for h in self.streams:
                if h != here:
                    cur = torch.cuda.current_stream()
                    cur.wait_stream(torch.cuda.ExternalStream(h))
                    for g in gs:
                        for t in ((g.grad, g.bits) if isinstance(g, MaskedGrad) else (g,)):
                            if isinstance(t, torch.Tensor) and t.is_cuda:
                                t.record_stream(cur)
            self.streams = []

    def take2(self):
        """Consumer side: both stashed gradients (either may be None), marking the consumer done."""
        g, g2 = self.grad, self.grad2
        self.grad = self.grad2 = None
        self.consumer_done = True
        self._sync(*(t for t in (g, g2) if t is not None))
        return g, g2

    def take(self):
        """Consumer side: the (summed) stashed gradient or None, marking the consumer as done."""
        g, g2 = self.take2()
        if g2 is not None:
            g = g + g2
        return g


# ---- weight gradients on a side stream ------------------------------------------------------
# A layer's weight gradient is needed only by the optimizer (and the bucket all-reduce); its data
# gradient feeds the next BatchNorm backward pass. With the weight gradient written straight into
# ``.grad`` (grad_sink) it can run on a side HIP stream, concurrently with the HBM-bound BatchNorm
# passes and the data gradients of the layers below. The side stream waits for the origin stream
# at each launch (dy and x are ready), the caching allocator keeps dy / x alive until the side
# stream is done with them, and the origin stream waits for the side stream at the end of the
# backward pass (an autograd final callback) and before every gradient bucket's all-reduce
# (parallel.ddp). DV_WGRAD_SIDE=0 keeps every launch on the origin stream.
# DV_WGRAD_SIDE=0 keeps every launch on the origin stream, "3x3" moves only the im2col (R*S > 1)
# ones. Same-box, ResNet-50: origin stream 13,152 img/s, 3x3 only 13,342, every wgrad 13,837
# (profiles/wgrad_side_stream_ab.txt); MobileNet V1 lost 1.8 % with its pointwise wgrads moved (they
# overlap its HBM-bound depthwise / BN passes, nothing gains) and opts out (models/mobilenet.py).
_POLICY = _policy.side_policy()  # the A/B switches (deep_vision_amd/policy.py reads them all)
WGRAD_SIDE = _POLICY["wgrad_side"]
SIDE_COMM = _POLICY["comm"]
_SIDE = {"streams": {}, "active": None, "suspend": 0}  # active: (origin, side stream) of this backward


@contextlib.contextmanager
def no_wgrad_side():
    """Convolutions built inside keep their weight gradients on the origin stream (a model that
    forks its own branch streams: models/hourglass.py, where a fifth stream would share a hardware
    queue with the branches). DV_WGRAD_SIDE_OPTOUT=0 ignores it (same-box A/B)."""
    if not _SIDE_OPTOUT:
        yield
        return
    _SIDE["suspend"] += 1
    try:
        yield
    finally:
        _SIDE["suspend"] -= 1


_SIDE_OPTOUT = _POLICY["optout"]
# Captured steps with >= 8 hardware queues keep weight gradients on the origin stream: a graph
# whose side-stream branches land on hardware queues of their own replayed 24-35 % slower
# (ResNet-50 --graph 13,120 -> 10,010 img/s, YOLOv3 1,142 -> 750; profiles/wgrad_side_stream_ab.txt).
# With HIP's default 4 (what bench.py / launch.spawn leave to captured steps) the side stream is kept
# (YOLOv3 --graph +2 %, ResNet-50 +0.3 %). DV_WGRAD_SIDE_GRAPH=0 / 1 forces it.


def _queue_policy():
    """(under_dp, in_capture) from the process's hardware-queue count, resolved at the first conv
    (after HIP initialised: the queue count is fixed by then), not at import."""
    qp = _SIDE.get("qp")
    if qp is None:
        sp = _policy.side_policy()
        qp = _SIDE["qp"] = (sp["under_dp"], sp["in_capture"])
    return qp


def _capturing():
    return not _queue_policy()[1] and torch.cuda.is_current_stream_capturing()


def _side_stream(device):
    s = _SIDE["streams"].get(device)
    if s is None:
        s = _SIDE["streams"][device] = torch.cuda.Stream(device=device)
    return s


# Under a process group the side stream needs hardware queues of its own: with HIP's default 4 it
# shared the compute stream's queue beside RCCL's streams and serialised behind it (world-1 RCCL
# ResNet-50 13,000 -> 12,300 img/s); with GPU_MAX_HW_QUEUES >= 8 (policy.configure sets 8 for eager
# steps) it overlaps (12,960 -> 13,690). DV_WGRAD_SIDE_DP=0 / 1 forces it off / on.


def _dist_active():
    """True when a process group is up and the side stream must stay off (see _queue_policy)."""
    if _queue_policy()[0]:
        return False
    import torch.distributed as dist

    return dist.is_available() and dist.is_initialized()


def wgrad_side_join():
    """End of backward: the origin stream waits for every weight gradient queued on the side stream."""
    a = _SIDE["active"]
    if a is not None:
        _SIDE["active"] = None
        a[0].wait_stream(a[1])


def wgrad_side_comm_stream():
    """For a consumer of ``.grad`` mid-backward (a bucket all-reduce): the side stream, made to wait
    for the current stream, when weight gradients are queued on it (the consumer then issues from
    it: ordered after both streams' work so far, and the origin stream does not stall); else None."""
    a = _SIDE["active"]
    if a is None:
        return None
    side = a[1]
    cur = torch.cuda.current_stream(side.device)
    if SIDE_COMM == "flush":  # the current stream waits for the queued weight gradients instead
        cur.wait_stream(side)
        return None
    side.wait_stream(cur)
    return side


def _on_side(fn, device, *keep):
    origin = torch.cuda.current_stream(device)
    side = _side_stream(device)
    if _SIDE["active"] is None:
        _SIDE["active"] = (origin, side)
        torch.autograd.Variable._execution_engine.queue_callback(wgrad_side_join)
    side.wait_stream(origin)
    with torch.cuda.stream(side):
        fn()
    for t in keep:
        t.record_stream(side)


def _wgrad(x, dy, weight, Cg_x, G, stride, padding, dilation, out=None, reflect=False):
    """Weight gradient (OIHW fp32). With ``out`` the result is ADDED into ``out`` (live grad).
    ``reflect``: the forward padded by reflection (im2col taps outside the image are mirrored)."""
    N, _, H, W = x.shape
    O, Ig, R, S = weight.shape
    Og = O // G
    _, _, P, Q = dy.shape
    sh, sw = stride
    ph, pw = padding
    dh, dw = dilation
    if R == 1 and S == 1 and Cg_x == Ig and not reflect:  # GEMM layout == OIHW: accumulate straight into the grad
        buf = out if out is not None else torch.empty((O, Ig, 1, 1), dtype=F32, device=x.device)
        lib().conv_wgrad(ptr(x), ptr(dy), ptr(buf), N, H, W, Cg_x, ld_of(x), G, Og, P, Q, ld_of(dy), R, S, sh, sw,
                         ph, pw, dh, dw, 0, int(out is not None), 0, stream_handle())
        return buf
    # [G][Og][R][S][Cg] into the persistent zeroed workspace (split-K atomics, no memset), then
    # one pass to OIHW that re-zeroes the workspace as it reads it
    # (split-K through ordered slabs: the slab reduce writes OIHW directly and the workspace is
    # not touched -- csrc/conv_wgrad.hip slab_reduce_oirs_kernel)
    ws = _wgrad_workspace(G * Og * R * S * Cg_x, x.device)
    dW = out if out is not None else torch.empty((O, Ig, R, S), dtype=F32, device=x.device)
    L = lib()
    r = L.conv_wgrad(ptr(x), ptr(dy), ptr(ws), N, H, W, Cg_x, ld_of(x), G, Og, P, Q, ld_of(dy), R, S, sh, sw, ph, pw,
                     dh, dw, 0, 1, 0, stream_handle(), reflect=int(reflect), out=ptr(dW), out_ig=Ig,
                     out_accumulate=int(out is not None))
    if not (r & L.WGRAD_FINAL):
        L.wgrad_unprep(ptr(ws), ptr(dW), G, Og, Ig, R, S, Cg_x, 1.0, int(out is not None), 1, stream_handle())
    return dW


_WS = {}


def _wgrad_workspace(numel, device):
    """Zero-filled fp32 scratch per (device, stream), kept zero by its consumer (wgrad_unprep)."""
    key = (device, stream_handle())
    ws = _WS.get(key)
    if ws is None or ws.numel() < numel:
        ws = torch.zeros(max(numel, 1 << 20), dtype=F32, device=device)
        _WS[key] = ws
    return ws


class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding, dilation, groups, act, slope, want_stats, stats_buf=None,
                extra=(0, 0), join=None, join_role=None, reflect=False, out_box=None, residual=None, residual_join=None,
                bias_via_bn=False, bias_colsum=None):
        ctx.colsum_box = bias_colsum
        R_, S_ = weight.shape[2], weight.shape[3]
        # under a process group only with >= 8 hardware queues (_SIDE_DP). Never with a residual
        # epilogue: its dy is handed on (dres / residual_join) to a consumer that may overwrite it in
        # place on the origin stream (a BN backward folding the stashed gradient, dx = xg) while the
        # side-stream weight gradient still reads it; record_stream only guards the free, not the write.
        ctx.wside = (bool(WGRAD_SIDE) and _SIDE["suspend"] == 0 and (WGRAD_SIDE == "all" or R_ * S_ > 1)
                     and residual is None and not _dist_active() and not _capturing())
        N, Cx, H, W = x.shape
        O, Ig, R, S = weight.shape
        G = groups
        Og = O // G
        ldx = ld_of(x)
        Cg_x = _gather_channels(x, Cx // G, G)  # padded channels (G == 1) are zeros
        P, Q = out_size(H + extra[0], W + extra[1], R, S, stride, padding, dilation)
        wk = _prep_weight(weight, G, Cg_x, mode=0)
        if out_box:  # write-into-slice: the epilogue stores into a channel slice of a concat buffer
            y = out_box[0]
            if (tuple(y.shape) != (N, O, P, Q) or not is_nhwc(y) or ld_of(y) % 8 or y.data_ptr() % 16):
                raise ValueError(f"conv2d out= must be an NHWC bf16 (slice) view of shape {(N, O, P, Q)}")
        else:
            y = empty_nhwc(N, O, P, Q, x.device)
        stats = None
        if want_stats:
            stats = stats_buf if stats_buf is not None else torch.zeros((STAT_ROWS, O), dtype=F32, device=x.device)
        b = bias.detach().float().contiguous() if bias is not None else None
        # residual: y = conv + b + residual in the store epilogue (same NHWC layout as y)
        ks = 1 if reflect else conv_ksplit(N * P * Q, Og, R * S * Cg_x, G)
        conv_fwd_raw(x, wk, y, b, stats, N, H, W, Cg_x, ldx, G, Og, P, Q, R, S, stride, padding, dilation,
                     act=act, slope=slope, reflect=reflect, res=residual, ksplit=ks)
        ctx.has_residual = residual is not None
        ctx.rjoin = residual_join  # the residual's gradient (= dy) is stashed there for its other consumer
        ctx.save_for_backward(x, weight, y if act else None)
        ctx.bias_param = bias  # leaf parameter (not saved): its gradient may sink in place
        # bias_via_bn: y feeds a training BatchNorm that returns this bias's gradient itself
        # (ops.bn, from its backward sums: no reduction pass over dy here)
        ctx.cfg = (stride, padding, dilation, G, act, slope, Cg_x, bias is not None and not bias_via_bn)
        ctx.reflect = reflect
        ctx.join = (join, join_role)
        # the producing BatchNorm of x: its backward statistics can ride on this conv's dgrad
        ctx.bnref = getattr(x, "_dv_bnref", None) if join_role != "producer" else None
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the statistics output
        if bias_via_bn and bias is not None:
            y._dv_bias_via_bn = True  # the consumer BN owes this bias's gradient (ops.bn.conv_bn_act)
        if want_stats:
            ctx.mark_non_differentiable(stats)
            return y, stats
        return y

    @staticmethod
    def backward(ctx, dy, *unused):
        x, weight, y = ctx.saved_tensors
        stride, padding, dilation, G, act, slope, Cg_x, has_bias = ctx.cfg
        if dy is None:
            join, role = ctx.join
            if join is not None and role == "consumer":
                g = join.take()  # nothing to add to: hand a stashed shortcut gradient through
                if isinstance(g, MaskedGrad):
                    g = g.materialize()
                return (g, None, None) + (None,) * 17
            return (None,) * 20
        dy = grad_nhwc(dy)
        if act:  # y and dy may be channel-slice views of concat buffers: strided rows kernel
            dy = act_grad(dy, y, act, slope)
        dx = dw = db = None
        join, role = ctx.join
        if ctx.needs_input_grad[0]:
            accum = join.take() if (join is not None and role == "consumer") else None
            if ctx.reflect:
                dx = _reflect_dgrad(dy, weight, x, Cg_x, G, stride, padding, dilation)
            else:
                dx = _dgrad(dy, weight, x.shape, Cg_x, G, stride, padding, dilation, x.device, accum=accum,
                            bnref=ctx.bnref)
            if dx.shape[1] != x.shape[1]:
                dx = dx[:, : x.shape[1]]
            if join is not None and role == "producer":
                dx = join.produce(dx)
        if ctx.needs_input_grad[1]:
            sink = grad_sink(weight)
            if sink is not None and ctx.wside and dy.is_cuda:
                _on_side(lambda: _wgrad(x, dy, weight, Cg_x, G, stride, padding, dilation, out=sink,
                                        reflect=ctx.reflect), dy.device, x, dy)
            else:
                dw = _wgrad(x, dy, weight, Cg_x, G, stride, padding, dilation, out=sink, reflect=ctx.reflect)
            if sink is not None:
                dw = None
        if has_bias and ctx.needs_input_grad[2]:
            db = _bias_grad(ctx.bias_param, dy, ctx.colsum_box)
        dres = dy if ctx.has_residual and ctx.needs_input_grad[16] else None  # y = ... + residual
        if dres is not None and ctx.rjoin is not None:
            dres = ctx.rjoin.produce(dres)
        return dx, dw, db, None, None, None, None, None, None, None, None, None, None, None, None, None, dres, None, None, None


# ---------------------------------------------------------------------------------------
# Tap-packed stem convolution: first layers with <= 4 input channels (ResNet/Inception 7x7 s2,
# AlexNet 11x11 s4, Hourglass 7x7 s2, ...). The input is re-laid out ONCE as a zero-padded
# [N][Hp][Wp][4] bf16 image; the kernel reads it as 8-tap x 4-channel rows (Cg = 4*Sp at a pixel
# stride of 4), so K = R * Sp * 4 (7x7: 224) instead of R * S * 8 with channels padded to 8
# (392): 1.75x fewer MFMA k-steps and no im2col bounds checks (csrc/conv_fwd.hip packed mode).
# ---------------------------------------------------------------------------------------
STEM_KERNELS = True  # 7x7 / 64-channel stems on csrc/stem.hip (else the packed implicit-GEMM path)
COUNTERS = {"stem_kernel_fwd": 0, "stem_generic_fwd": 0, "stem_kernel_wgrad": 0}


def _stem_geometry(x, weight, stride, padding, dilation, groups, extra):
    """(Sp, Hp, Wp, P, Q) when the tap-packed path applies, else None."""
    if groups != 1 or tuple(dilation) != (1, 1) or x.requires_grad or x.dim() != 4 or x.dtype not in (F32, BF16):
        return None
    N, C, H, W = x.shape
    O, I, R, S = weight.shape
    if C > 4 or I != C or stride[1] % 2 or not (5 <= S <= 16) or R > 16 or min(padding) < 0:
        return None
    Sp = 8 if S <= 8 else 16
    P, Q = out_size(H + extra[0], W + extra[1], R, S, stride, padding, dilation)
    Hp = (P - 1) * stride[0] + R
    Wp = (Q - 1) * stride[1] + Sp  # even: every 16-B chunk starts at an even pixel
    return Sp, Hp, Wp, P, Q


def _prep_stem_weight(weight, Sp):
    O, I, R, S = weight.shape
    n = O * R * Sp * 4

    def compute(out):
        w = weight.detach()
        if w.dtype != F32 or not w.is_contiguous():
            w = w.float().contiguous()
        if out is None:
            out = torch.empty(n, dtype=BF16, device=w.device)
        lib().wprep(ptr(w), ptr(out), 1, O, I, R, S, 4, 2, Sp, stream_handle())
        return out

    if isinstance(weight, torch.nn.Parameter) and weight.dtype == F32 and weight.is_contiguous():
        return wcache.get(weight, 1, 4, 2, compute, Sp=Sp)
    return compute(None)


class _StemConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding, act, slope, want_stats, stats_buf, geo, reflect=False):
        Sp, Hp, Wp, P, Q = geo
        N, C, H, W = x.shape
        O, I, R, S = weight.shape
        xc = x if x.is_contiguous() else x.contiguous()
        xp = torch.empty((N, Hp, Wp, 4), dtype=BF16, device=x.device)
        lib().stem_pack(ptr(xc), int(xc.dtype == F32), ptr(xp), N, C, H, W, Hp, Wp, padding[0], padding[1],
                        stream_handle(), reflect=int(reflect))
        wk = _prep_stem_weight(weight, Sp)
        y = empty_nhwc(N, O, P, Q, x.device)
        stats = None
        if want_stats:
            stats = stats_buf if stats_buf is not None else torch.zeros((STAT_ROWS, O), dtype=F32, device=x.device)
        b = bias.detach().float().contiguous() if bias is not None else None
        r = -1
        if STEM_KERNELS and act in (0, 1, 2):  # dedicated row-walking 7x7 / 64-channel kernel (csrc/stem.hip)
            r = lib().stem_fwd(ptr(xp), ptr(wk), ptr(y), ptr(b), ptr(stats), int(act), float(slope), N, Hp, Wp, P, Q,
                               R, Sp, O, stride[0], stride[1], stream_handle())
        if r != 0:
            conv_fwd_raw(xp, wk, y, b, stats, N, Hp, Wp, 4 * Sp, 4, 1, O, P, Q, R, 1, stride, (0, 0), (1, 1), act=act,
                         slope=slope, tgather=2)
        COUNTERS["stem_kernel_fwd" if r == 0 else "stem_generic_fwd"] += 1
        ctx.save_for_backward(xp, weight, y if act else None)
        ctx.bias_param = bias  # leaf parameter (not saved): its gradient may sink in place
        ctx.cfg = (stride, act, slope, geo, bias is not None)
        ctx.set_materialize_grads(False)
        if want_stats:
            ctx.mark_non_differentiable(stats)
            return y, stats
        return y

    @staticmethod
    def backward(ctx, dy, *unused):
        xp, weight, y = ctx.saved_tensors
        stride, act, slope, geo, has_bias = ctx.cfg
        if dy is None:
            return (None,) * 11
        Sp, Hp, Wp, P, Q = geo
        O, I, R, S = weight.shape
        N = xp.shape[0]
        dy = grad_nhwc(dy)
        if act:
            dy = act_grad(dy, y, act, slope)
        dw = db = None
        if ctx.needs_input_grad[1] and STEM_KERNELS and not lib().deterministic():
            # dedicated kernel: per-block partials reduced straight into the [O][C][R][S] gradient
            sink = grad_sink(weight)
            dst = sink if sink is not None else torch.zeros(weight.shape, dtype=F32, device=xp.device)
            r = lib().stem_wgrad(ptr(xp), ptr(dy), ld_of(dy), ptr(dst), N, I, S, Hp, Wp, P, Q, R, Sp, O, stride[0],
                                 stride[1], stream_handle())
            if r == 0:
                COUNTERS["stem_kernel_wgrad"] += 1
                if sink is None:
                    dw = dst
                if has_bias and ctx.needs_input_grad[2]:
                    db = _bias_grad(ctx.bias_param, dy)
                return None, dw, db, None, None, None, None, None, None, None, None
            if sink is None:
                del dst
        if ctx.needs_input_grad[1]:
            ws = _wgrad_workspace(O * R * Sp * 4, xp.device)  # [O][R][Sp][4], zero on entry and exit
            lib().conv_wgrad(ptr(xp), ptr(dy), ptr(ws), N, Hp, Wp, 4 * Sp, 4, 1, O, P, Q, ld_of(dy), R, 1, stride[0],
                             stride[1], 0, 0, 1, 1, 0, 1, 0, stream_handle())
            full = torch.empty((O, I, R, Sp), dtype=F32, device=xp.device)
            lib().wgrad_unprep(ptr(ws), ptr(full), 1, O, I, R, Sp, 4, 1.0, 0, 1, stream_handle())
            sink = grad_sink(weight)
            if sink is not None:
                sink.add_(full[..., :S])
            else:
                dw = full[..., :S].contiguous()
        if has_bias and ctx.needs_input_grad[2]:
            db = _bias_grad(ctx.bias_param, dy)
        return None, dw, db, None, None, None, None, None, None, None, None


def conv2d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, act=None, slope=0.0,
           want_stats=False, stats_buf=None, join=None, join_role=None, pad_mode="zeros", out=None, residual=None,
           residual_join=None, shuffle=0, bias_via_bn=False, bias_colsum=None):
    """Conv2d (+fused bias/activation). Returns y, or (y, stats) when want_stats (GPU only).

    ``bias_colsum`` (ColsumBox): the BN consuming y sums y's gradient per channel in its backward
    apply pass; the bias gradient is folded from those sums (models/hourglass.py).

    ``shuffle=g`` (> 1): the output channels are channel-shuffled in g groups (ShuffleNet V1;
    fused into the grouped 1x1 kernel's store on the native path, csrc/gconv.hip).

    ``padding`` may be (top, bottom, left, right) for TF/Keras asymmetric 'same' padding.
    ``pad_mode='reflect'``: ReflectionPad2d(padding) fused into the im2col gather (the taps
    outside the image read the mirrored pixels; no padded copy of the input).
    ``out``: a preallocated NHWC (channel-slice) view the output is written into (write-into-slice
    concat, ops.concat.slice_cat); native path only.
    ``residual``: y = conv(x) + bias + residual, the add fused into the store epilogue (no
    activation / statistics; Hourglass bottleneck output, R/Hourglass/tensorflow/hourglass104.py:62-67)."""
    if shuffle and shuffle > 1:
        if native(x) and _gconv_ok(x, weight, bias, stride, padding, dilation, groups, act, join=join, out=out,
                                   residual=residual, pad_mode=pad_mode):
            return _gconv(x, weight, groups, shuffle, want_stats, stats_buf)
        from .concat import channel_shuffle

        # no statistics from the inner conv: they would land in the BN's workspace in the
        # unshuffled channel order, and the BN takes its own pass over the shuffled output
        y = conv2d(x, weight, bias, stride, padding, dilation, groups, act, slope, False, None, join,
                   join_role, pad_mode, out, residual, residual_join)
        y = channel_shuffle(y, shuffle)
        return (y, None) if want_stats else y
    # want_stats with a residual: statistics of the final y = conv + bias + residual (the conv
    # epilogue accumulates them from its stores; a pre-activation block output feeding a BN)
    res_stats_ok = (want_stats and native(x) and not act and out is None and groups == 1 and pad_mode == "zeros"
                    and weight.shape[0] % 8 == 0)
    if residual is not None and (act or (want_stats and not res_stats_ok) or out is not None or not native(x)):
        y = conv2d(x, weight, bias, stride, padding, dilation, groups, act, slope, False, None, join,
                   join_role, pad_mode, out)
        y = y + residual if not native(x) else _add_native(y, residual)
        return (y, None) if want_stats else y
    if isinstance(padding, str):
        raise NotImplementedError("string padding: use nn.Conv2d(padding='same_keras')")
    stride, dilation = _pair(stride), _pair(dilation)
    padding, extra = norm_padding(padding)
    reflect = pad_mode == "reflect"
    if pad_mode not in ("zeros", "reflect"):
        raise NotImplementedError(f"pad_mode {pad_mode!r}")
    if reflect and (extra != (0, 0) or dilation != (1, 1)):
        raise NotImplementedError("reflect padding with asymmetric pads / dilation")
    if join is not None and join_role == "consumer" and (not native(x) or reflect):
        join.consumer_done = True
    if reflect:
        join = None
    if not native(x):
        if reflect:
            x = TF.pad(x, (padding[1], padding[1], padding[0], padding[0]), mode="reflect")
            padding = (0, 0)
        if extra != (0, 0):
            x = TF.pad(x, (padding[1], padding[1] + extra[1], padding[0], padding[0] + extra[0]))
            padding = (0, 0)
        y = TF.conv2d(x, weight, bias, stride, padding, dilation, groups)
        if act in ("relu",):
            y = TF.relu(y)
        elif act in ("leaky", "leaky_relu"):
            y = TF.leaky_relu(y, slope)
        return (y, None) if want_stats else y
    dw = _is_depthwise(x, weight, groups, stride, dilation)
    padded_groups = groups > 1 and ((x.shape[1] // groups) % 8 != 0 or (weight.shape[0] // groups) % 8 != 0)
    if join is not None and join_role == "consumer" and dw:
        join.consumer_done = True  # the depthwise path does not fold the join: producers hand grads to autograd
    if reflect and dw:
        raise NotImplementedError("reflect padding on depthwise convs")
    if out is not None and (dw or padded_groups):
        raise NotImplementedError("conv2d out= on depthwise / channel-padded grouped convs")
    if dw:
        return depthwise_conv2d(x, weight, bias, stride, padding, act, slope, want_stats, stats_buf, extra)
    if padded_groups and _gconv_ok(x, weight, bias, stride, padding, dilation, groups, act, join=join, out=out,
                                   residual=residual, pad_mode=pad_mode):
        # channels per group not a multiple of 8 (ShuffleNet V1 g=3: 20 per group): the grouped
        # 1x1 kernel (csrc/gconv.hip) -- per-group MFMA tiles, no block-diagonal expansion
        return _gconv(x, weight, groups, 0, want_stats, stats_buf)
    if padded_groups:
        # other shapes (k > 1, strided): a dense conv with a block-diagonal weight
        weight = _block_diagonal(weight, groups, x.shape[1])
        groups = 1
    geo = _stem_geometry(x, weight, stride, padding, dilation, groups, extra)
    if geo is not None:  # network input: no gradient, no join
        if join is not None and join_role == "consumer":
            join.consumer_done = True
        return _StemConvFn.apply(x, weight, bias, stride, padding, ACT_IDS[act], float(slope), want_stats, stats_buf,
                                 geo, reflect)
    xn = as_nhwc(x, pad_to8=(groups == 1))
    if xn is not x and join is not None:
        if join_role == "consumer":  # the gradient reaches x through the layout copy: no join
            join.consumer_done = True
        join = None
    res = None
    if residual is not None:
        if not (dw or padded_groups or geo is not None):
            res = as_nhwc(residual, pad_to8=True)
            if ld_of(res) != round8(weight.shape[0]) or res.data_ptr() % 16:
                res = (res.contiguous(memory_format=torch.channels_last) if round8(weight.shape[0]) == weight.shape[0]
                       else None)
        if res is None:  # the add as its own pass (no statistics from it)
            y = _add_native(conv2d(x, weight, bias, stride, padding, dilation, groups, act, slope, False, None, join,
                                   join_role, pad_mode, out), residual)
            return (y, None) if want_stats else y
    if res is None:
        residual_join = None
    return _CONV_APPLY(xn, weight, bias, stride, padding, dilation, groups, ACT_IDS[act], float(slope), want_stats,
                         stats_buf, extra, join, join_role, reflect, [out] if out is not None else None, res,
                         residual_join, bool(bias_via_bn and bias is not None and not act), bias_colsum)


def _gconv_ok(x, weight, bias, stride, padding, dilation, groups, act, join=None, out=None, residual=None,
              pad_mode="zeros"):
    """Shapes the grouped 1x1 kernel serves: 1x1, stride 1, no padding / bias / activation /
    residual / concat slice, 4-aligned channels per group (wgrad register blocks)."""
    O, Cg, R, S = weight.shape
    C = x.shape[1]
    return (R == 1 and S == 1 and _pair(stride) == (1, 1) and _pair(dilation) == (1, 1)
            and all(v == 0 for v in norm_padding(padding)[0]) and norm_padding(padding)[1] == (0, 0)
            and bias is None and not act and out is None and residual is None and pad_mode == "zeros" and join is None
            and C == Cg * groups and O % groups == 0 and Cg % 4 == 0 and (O // groups) % 4 == 0 and x.dim() == 4)


_PERM = {}


def _shuffle_table(C, sg, device):
    """int16 logical -> stored channel table of the ShuffleNet shuffle (None = identity)."""
    if not sg or sg <= 1:
        return None
    key = (C, sg, str(device))
    t = _PERM.get(key)
    if t is None:
        l = torch.arange(C)
        cpg = C // sg
        t = _PERM[key] = ((l % cpg) * sg + l // cpg).to(torch.int16).to(device)
    return t


class _GConvFn(torch.autograd.Function):
    """Grouped 1x1 conv (+ fused output channel shuffle, + BN statistics) on csrc/gconv.hip."""

    @staticmethod
    def forward(ctx, x, weight, groups, shuffle, want_stats, stats_buf):
        N, C, H, W = x.shape
        O, Cg = weight.shape[0], weight.shape[1]
        G, Og = groups, weight.shape[0] // groups
        Kp = (Cg + 31) // 32 * 32
        wk = _prep_weight(weight, G, Kp, mode=0)  # [G][Og][Kp]
        y = empty_nhwc(N, O, H, W, x.device)
        stats = None
        if want_stats:
            stats = stats_buf if stats_buf is not None else torch.zeros((STAT_ROWS, O), dtype=F32, device=x.device)
        tab = _shuffle_table(O, shuffle, x.device)
        lib().gconv(ptr(x), ld_of(x), C, 0, ptr(wk), Og, ptr(y), ld_of(y), O, ptr(tab), N * H * W, G, Cg, Og, Kp,
                    ptr(stats), stream_handle())
        ctx.save_for_backward(x, weight)
        ctx.cfg = (G, int(shuffle))
        ctx.set_materialize_grads(False)
        if want_stats:
            ctx.mark_non_differentiable(stats)
            return y, stats
        return y

    @staticmethod
    def backward(ctx, dy, *unused):
        x, weight = ctx.saved_tensors
        G, sg = ctx.cfg
        if dy is None:
            return (None,) * 6
        dy = grad_nhwc(dy)
        if dy.data_ptr() % 16:
            dy = dy.contiguous(memory_format=torch.channels_last)
        N, C, H, W = x.shape
        O, Cg = weight.shape[0], weight.shape[1]
        Og = O // G
        dx = dw = None
        if ctx.needs_input_grad[0]:
            Kp = (Og + 31) // 32 * 32
            wt = _prep_weight(weight, G, Kp, mode=1)  # [G][Cg][Kp]: per-group transpose
            dx = empty_nhwc(N, C, H, W, x.device)
            lib().gconv(ptr(dy), ld_of(dy), O, ptr(_shuffle_table(O, sg, x.device)), ptr(wt), Cg, ptr(dx), ld_of(dx), C,
                        0, N * H * W, G, Og, Cg, Kp, 0, stream_handle())
        if ctx.needs_input_grad[1]:
            sink = grad_sink(weight)
            acc = sink if sink is not None else torch.zeros(weight.shape, dtype=F32, device=x.device)
            lib().gconv_wgrad(ptr(x), ld_of(x), 0, ptr(dy), ld_of(dy), ptr(_shuffle_table(O, sg, x.device)), ptr(acc),
                              N * H * W, G, Cg, Og, stream_handle())
            dw = None if sink is not None else acc
        return dx, dw, None, None, None, None


def _gconv(x, weight, groups, shuffle, want_stats, stats_buf):
    C = x.shape[1]
    xn = as_nhwc(x, pad_to8=True)
    if xn.shape[1] != C:  # as_nhwc padded the logical channels: keep the padded storage, view C
        xn = xn[:, :C]
    if xn.data_ptr() % 16 or ld_of(xn) < round8(C) or ld_of(xn) % 8:
        xn = empty_nhwc(*xn.shape, x.device)
        xn.copy_(x)
    return _GConvFn.apply(xn, weight, groups, shuffle, want_stats, stats_buf)


def _add_native(a, b):
    from .act import add

    return add(a, b)


def _block_diagonal(weight, groups, cin):
    """Grouped OIHW weight (O, C/G, R, S) -> the equivalent dense weight (O, C, R, S) with zeros
    outside each output channel's group (differentiable: gradients flow back to ``weight``)."""
    O, Cg, R, S = weight.shape
    Og = O // groups
    key = (O, cin, groups, str(weight.device))
    mask = _BD_MASK.get(key)
    if mask is None:
        o = torch.arange(O, device=weight.device) // Og
        c = torch.arange(cin, device=weight.device) // Cg
        mask = (o[:, None] == c[None, :]).to(weight.dtype)[:, :, None, None]
        _BD_MASK[key] = mask
    return weight.repeat(1, groups, 1, 1) * mask


_BD_MASK = {}


# ---------------------------------------------------------------------------------------
# ConvTranspose2d: forward = conv dgrad with the transposed-conv weight [Cin][Cout][R][S]
# ---------------------------------------------------------------------------------------
class _ConvTFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding, output_padding, dilation, groups, out_hw=None):
        # x (N, Cin, H, W), weight (Cin, Cout/G, R, S). Equivalent conv: W_conv = weight with
        # O := Cin, I := Cout/G; output = dgrad(x) of that conv with output size (OH, OW).
        # ``out_hw`` overrides the output size (Keras 'same': H*stride with a top/left pad of
        # (k - s) // 2, i.e. the torch result cropped at the bottom/right).
        N, Cin, H, W = x.shape
        Ci, Cog, R, S = weight.shape
        G = groups
        sh, sw = stride
        ph, pw = padding
        dh, dw = dilation
        OH = (H - 1) * sh - 2 * ph + dh * (R - 1) + output_padding[0] + 1
        OW = (W - 1) * sw - 2 * pw + dw * (S - 1) + output_padding[1] + 1
        if out_hw is not None:
            OH, OW = out_hw
        Cout = Cog * G
        if G > 1 and (Cog % 8 != 0):
            raise NotImplementedError("grouped ConvTranspose requires out-channels-per-group % 8 == 0")
        # The transposed-conv weight [Cin][Cog][R][S] is a conv weight with O = Cin, I = Cog;
        # its forward is that conv's dgrad: operand [G][Cog][R][S][Cin/G] (wprep mode 1).
        Cpad = round8(Cog) if G == 1 else Cog
        Cg_in = _gather_channels(x, Ci // G, G)
        wd = _prep_weight(weight, G, Cg_in, mode=1)
        y_full = alloc_cl((N, G * Cpad, OH, OW), zero=(Cpad != Cog), device=x.device)
        ldx = ld_of(x)
        b = bias.detach().float().contiguous() if bias is not None else None  # bias in the epilogue
        if (sh, sw) == (1, 1):
            conv_fwd_raw(x, wd, y_full, b, None, N, H, W, Cg_in, ldx, G, Cog, OH, OW, R, S, (1, 1), (-ph, -pw),
                         (-dh, -dw), ldy=G * Cpad)
        else:
            conv_fwd_raw(x, wd, y_full, b, None, N, H, W, Cg_in, ldx, G, Cog, OH, OW, R, S, stride, padding,
                         dilation, tgather=1, ldy=G * Cpad)
        y = y_full if Cpad == Cog else y_full[:, :Cout]
        ctx.save_for_backward(x, weight)
        ctx.bias_param = bias  # leaf parameter (not saved): its gradient may sink in place
        ctx.cfg = (stride, padding, dilation, G, bias is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        stride, padding, dilation, G, has_bias = ctx.cfg
        dy = grad_nhwc(dy)
        Ci, Cog, R, S = weight.shape
        N, Cin, H, W = x.shape
        dx = dw = db = None
        Cg_dy = _gather_channels(dy, Cog, G)
        if ctx.needs_input_grad[0]:
            # dX = conv_fwd(dY, W_conv) with W_conv[o = Cin][i = Cog]
            wk = _prep_weight(weight, G, Cg_dy, mode=0)
            dx = empty_nhwc(N, Cin, H, W, x.device)
            conv_fwd_raw(dy, wk, dx, None, None, N, dy.shape[2], dy.shape[3], Cg_dy, ld_of(dy), G, Ci // G, H, W, R, S,
                         stride, padding, dilation)
        if ctx.needs_input_grad[1]:
            # conv relationship: X_conv = dY (large), dY_conv = x (small)
            dw = _wgrad(dy, x, weight, Cg_dy, G, stride, padding, dilation)
        if has_bias and ctx.needs_input_grad[2]:
            db = _bias_grad(ctx.bias_param, dy)
        return dx, dw, db, None, None, None, None, None, None


def keras_same_transpose(H, W, kernel_size, stride):
    """Keras Conv2DTranspose(padding='same'): output (H*s, W*s), top/left pad (k - s) // 2."""
    (kh, kw), (sh, sw) = _pair(kernel_size), _pair(stride)
    return (max(kh - sh, 0) // 2, max(kw - sw, 0) // 2), (H * sh, W * sw)


def conv_transpose2d(x, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1, dilation=1,
                     output_size=None):
    """torch.nn.functional.conv_transpose2d; ``output_size=(OH, OW)`` crops / fixes the output
    grid (used for Keras 'same' transposed convs whose size torch cannot express)."""
    stride, padding, output_padding, dilation = _pair(stride), _pair(padding), _pair(output_padding), _pair(dilation)
    if not native(x):
        if output_size is None:
            return TF.conv_transpose2d(x, weight, bias, stride, padding, output_padding, groups, dilation)
        y = TF.conv_transpose2d(x, weight, bias, stride, 0, 0, groups, dilation)
        return y[:, :, padding[0]:padding[0] + output_size[0], padding[1]:padding[1] + output_size[1]]
    x = as_nhwc(x, pad_to8=(groups == 1))
    return _ConvTFn.apply(x, weight, bias, stride, padding, output_padding, dilation, groups,
                          tuple(output_size) if output_size is not None else None)


# ---------------------------------------------------------------------------------------
# Linear: a 1x1 conv over an (N, K) "image" of one pixel
# ---------------------------------------------------------------------------------------
class _LinearFn(torch.autograd.Function):
    """y = x W^T + b as a 1x1 conv over N one-pixel images (rows)."""

    @staticmethod
    def forward(ctx, x, weight, bias, act, slope):
        N, K = x.shape
        O, _ = weight.shape
        Kp = x.stride(0)  # zero-padded row stride, multiple of 8
        wk = _prep_weight(weight.view(O, K, 1, 1), 1, Kp, mode=0, param=weight)
        Op = round8(O)
        y_full = (torch.zeros if Op != O else torch.empty)((N, Op), dtype=BF16, device=x.device)
        b = bias.detach().float().contiguous() if bias is not None else None
        conv_fwd_raw(x, wk, y_full, b, None, N, 1, 1, Kp, Kp, 1, O, 1, 1, 1, 1, (1, 1), (0, 0), (1, 1), act=act,
                     slope=slope, ldy=Op, ksplit=gemm_ksplit(N, O, Kp))
        y = y_full if Op == O else y_full[:, :O]
        ctx.save_for_backward(x, weight, bias, y if act else None)
        ctx.bias_param = bias  # leaf parameter (not saved): its gradient may sink in place
        ctx.cfg = (act, slope, bias is not None, Kp, Op)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, bias, y = ctx.saved_tensors
        act, slope, has_bias, Kp, Op = ctx.cfg
        N, K = x.shape
        O, _ = weight.shape
        if dy.dtype != BF16 or dy.stride(1) != 1 or dy.stride(0) != Op:
            g = (torch.zeros if Op != O else torch.empty)((N, Op), dtype=BF16, device=dy.device)
            g[:, :O].copy_(dy)
            dy = g[:, :O]
        if act:
            g = (torch.zeros if Op != O else torch.empty)((N, Op), dtype=BF16, device=dy.device)
            lib().act_bwd(ptr(dy), ptr(y), ptr(g), N * Op, act, float(slope), stream_handle())
            dy = g[:, :O]
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            wd = _prep_weight(weight.view(O, K, 1, 1), 1, Op, mode=1, param=weight)  # [K][Op]
            dx_full = (torch.zeros if Kp != K else torch.empty)((N, Kp), dtype=BF16, device=dy.device)
            conv_fwd_raw(dy, wd, dx_full, None, None, N, 1, 1, Op, Op, 1, K, 1, 1, 1, 1, (1, 1), (0, 0), (1, 1),
                         ldy=Kp, ksplit=gemm_ksplit(N, K, Op))
            dx = dx_full if Kp == K else dx_full[:, :K]
        if ctx.needs_input_grad[1]:
            sink = grad_sink(weight)
            buf = sink if sink is not None else torch.empty((O, K), dtype=F32, device=dy.device)
            lib().conv_wgrad(ptr(x), ptr(dy), ptr(buf), N, 1, 1, Kp, Kp, 1, O, 1, 1, Op, 1, 1, 1, 1, 0, 0, 1, 1, 0,
                             int(sink is not None), K if Kp != K else 0, stream_handle())
            if sink is not None:
                dw = None
            else:
                dw = buf
        if has_bias and ctx.needs_input_grad[2]:
            # native per-column sum of the bf16 rows, added straight into the live gradient buffer
            # when there is one (instead of a bf16->fp32 copy + reduce + autograd add)
            sink = grad_sink(ctx.bias_param)
            key = (str(dy.device), Op)
            acc = _CSUM_WS.get(key)
            if acc is None:
                acc = _CSUM_WS[key] = torch.zeros((STAT_ROWS, Op), dtype=F32, device=dy.device)
            dst = sink if sink is not None else torch.empty(O, dtype=F32, device=dy.device)
            lib().channel_sum(ptr(dy), N, Op, O, ptr(acc), ptr(dst), int(sink is not None), stream_handle())
            db = None if sink is not None else dst
        return dx, dw, db, None, None


def linear(x, weight, bias=None, act=None, slope=0.0):
    if not native(x):
        y = TF.linear(x, weight, bias)
        if act == "relu":
            y = TF.relu(y)
        elif act in ("leaky", "leaky_relu"):
            y = TF.leaky_relu(y, slope)
        return y
    lead = x.shape[:-1]
    x2 = x.reshape(-1, x.shape[-1])
    K = x2.shape[1]
    if x2.dtype != BF16 or x2.stride(1) != 1 or x2.stride(0) % 8 != 0 or x2.stride(0) < K:
        Kp = round8(K)
        xp = (torch.zeros if Kp != K else torch.empty)((x2.shape[0], Kp), dtype=BF16, device=x.device)
        if x2.requires_grad:
            xp = TF.pad(x2.to(BF16), (0, Kp - K)) if Kp != K else x2.to(BF16).contiguous()
        else:
            xp[:, :K].copy_(x2)
        x2 = xp if Kp == K else xp[:, :K]
    y = _LinearFn.apply(x2, weight, bias, ACT_IDS[act], float(slope))
    return y.reshape(*lead, weight.shape[0])


# ---------------------------------------------------------------------------------------
# Depthwise conv (groups == in == out channels): csrc/depthwise.hip
# ---------------------------------------------------------------------------------------
class _DWConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding, act, slope, want_stats, stats_buf, extra=(0, 0)):
        N, C, H, W = x.shape
        K = weight.shape[2]
        P, Q = out_size(H + extra[0], W + extra[1], K, K, stride, padding, (1, 1))
        y = empty_nhwc(N, C, P, Q, x.device)
        w = weight.detach().float().contiguous()
        b = bias.detach().float().contiguous() if bias is not None else None
        stats = None
        if want_stats:
            stats = stats_buf if stats_buf is not None else torch.zeros((STAT_ROWS, C), dtype=F32, device=x.device)
        lib().dw_fwd(ptr(x), ptr(w), ptr(b), ptr(y), N, H, W, C, ld_of(x), P, Q, ld_of(y), K, stride[0], stride[1],
                     padding[0], padding[1], act, float(slope), ptr(stats), stream_handle())
        ctx.save_for_backward(x, weight, y if act else None)
        ctx.bias_param = bias  # leaf parameter (not saved): its gradient may sink in place
        ctx.cfg = (stride, padding, act, slope, bias is not None)
        # x is a BatchNorm output (MobileNet: pw -> BN -> ReLU -> dw): its backward reduction is
        # folded into this dgrad's epilogue (modes 1 / 2: no mask bits), cf. _ConvFn
        # (stride 1 only: the stride-2 dgrad writes 4x the pixels it reads, and reading the BN input
        # there as well cost as much as the separate reduce pass it saved, profiles/archive/dw_bench_r3b.txt)
        bnref = getattr(x, "_dv_bnref", None)
        ctx.bnref = (bnref if (bnref is not None and bnref.mode in (1, 2) and ld_of(x) == C and tuple(stride) == (1, 1))
                     else None)
        ctx.set_materialize_grads(False)
        if want_stats:
            ctx.mark_non_differentiable(stats)
            return y, stats
        return y

    @staticmethod
    def backward(ctx, dy, *unused):
        x, weight, y = ctx.saved_tensors
        stride, padding, act, slope, has_bias = ctx.cfg
        if dy is None:
            return (None,) * 10
        dy = grad_nhwc(dy)
        if act:
            dy = act_grad(dy, y, act, slope)
        N, C, H, W = x.shape
        K = weight.shape[2]
        P, Q = dy.shape[2], dy.shape[3]
        w = weight.detach().float().contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = empty_nhwc(N, C, H, W, x.device)
            br = ctx.bnref
            bn = {}
            if br is not None:
                bn = dict(bnx=ptr(br.x), bnprm=ptr(br.prm), bnacc=ptr(br.acc), bnmode=br.mode, bnact=br.act,
                          bnslope=float(br.slope))
            lib().dw_dgrad(ptr(dy), ptr(w), ptr(dx), N, H, W, C, ld_of(dx), P, Q, ld_of(dy), K, stride[0], stride[1],
                           padding[0], padding[1], stream_handle(), **bn)
            if br is not None:
                br.mark_fused(dx)
        if ctx.needs_input_grad[1]:
            sink = grad_sink(weight)
            buf = sink if sink is not None else torch.empty_like(w)
            lib().dw_wgrad(ptr(x), ptr(dy), ptr(buf), N, H, W, C, ld_of(x), P, Q, ld_of(dy), K, stride[0], stride[1],
                           padding[0], padding[1], int(sink is not None), stream_handle())
            if sink is None:
                dw = buf
        if has_bias and ctx.needs_input_grad[2]:
            db = _bias_grad(ctx.bias_param, dy)
        return dx, dw, db, None, None, None, None, None, None, None


def _is_depthwise(x, weight, groups, stride, dilation):
    O, Ig, R, S = weight.shape
    # the dgrad kernels cover strides (1, 1) and (2, 2) only (csrc/depthwise.hip dv_dw_dgrad):
    # anything else takes the grouped path instead of failing in backward
    return (groups > 1 and groups == x.shape[1] and O == groups and Ig == 1 and R == S and R in (1, 3, 5, 7)
            and dilation == (1, 1) and tuple(stride) in ((1, 1), (2, 2)) and x.shape[1] % 8 == 0)


def depthwise_conv2d(x, weight, bias=None, stride=1, padding=0, act=None, slope=0.0, want_stats=False,
                     stats_buf=None, extra=(0, 0)):
    stride, padding = _pair(stride), _pair(padding)
    x = as_nhwc(x, pad_to8=False)
    return _DWCONV_APPLY(x, weight, bias, stride, padding, ACT_IDS[act], float(slope), want_stats, stats_buf,
                           extra)


_CONV_APPLY = fast_apply(_ConvFn)
_DWCONV_APPLY = fast_apply(_DWConvFn)
