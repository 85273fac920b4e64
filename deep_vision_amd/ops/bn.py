"""BatchNorm2d (+ fused activation and residual add) on the native kernels (csrc/bn.hip).

Training forward  : statistics come from the producing conv's epilogue when available
                    (``conv2d(..., want_stats=True)``), otherwise from ``bn_stats``; one
                    ``bn_finalize`` launch computes mean / invstd / scale / shift and updates
                    running statistics; one ``bn_apply`` pass writes act(x*scale+shift(+res)).
Training backward : ``bn_bwd_reduce`` (sum dz, sum dz*xhat with the activation mask fused) ->
                    ``bn_bwd_finalize`` (dgamma, dbeta) -> ``bn_bwd_apply`` (dx, and dz for the
                    residual branch).
Eval              : scale/shift from running statistics, single apply pass.

Reference semantics: torch.nn.BatchNorm2d after every conv of the PT ResNet/MobileNet
(R/ResNet/pytorch/models/resnet50.py:30,110-134); Keras BatchNormalization for the TF-origin
models (eps 1e-3, momentum 0.99 -> PyTorch momentum 0.01; Hourglass 0.9 -> 0.1).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as TF

from .common import (ACT_IDS, BF16, F32, fast_apply, grad_nhwc, grad_sink, is_nhwc, ld_of, lib, native, ptr,
                     stream_handle, workspace)

STAT_SHARDS = 64
STAT_ROWS = 2 * STAT_SHARDS + 1  # forward statistics: shard sums + the shift row (csrc/kernels.h)
FUSE_BWD_STATS = True  # fold the backward reduction into the consumer conv's dgrad epilogue
LAZY_SHORTCUT = True   # identity-shortcut gradient masked inside the consumer's dgrad epilogue
FOLD_RESIDUAL_BN = True  # projection-shortcut BN applied inside the block's last BN pass
DUAL_BWD = True  # ...and its backward: reduction in the consumer dgrad's epilogue, one dual apply pass
# small BatchNorms (C % 64 == 0, <= 2M elements), eager steps: the statistics fold inside the apply
# passes instead of a separate finalize launch, forward and backward (csrc/bn.hip "Small BatchNorms")
FUSE_FINALIZE = os.environ.get("DV_FUSE_FIN", "1") != "0"
COUNTERS = {"bwd_reduce_fused": 0, "bwd_reduce_pass": 0, "shortcut_lazy": 0, "dual_apply": 0, "dual_fused": 0,
            "bwd_apply_two_addends": 0, "bn_fin_fused": 0, "bn_bwd_fin_fused": 0}


class BNRef:
    """What a consumer conv's dgrad needs to fold this BatchNorm's backward reduction (sum dz,
    sum dz*xhat) into its epilogue (csrc/conv_fwd.hip BNR): the BN input, mask source and
    statistics. Attached to the BN output tensor (``_dv_bnref``); the conv records the gradient
    tensor it produced, and the BN backward uses the fused sums only if the gradient it receives
    IS that tensor (same storage, untouched version, a single fusion) -- otherwise it zeroes the
    accumulator and runs its own reduce pass.
    ``x2, prm2, acc2``: a residual block's projection BN folded into this pass (mode 3, the same
    dz): the epilogue reduces it too (sum dz shared, its own sum dz*xhat2)."""

    __slots__ = ("x", "bits", "prm", "mode", "act", "slope", "acc", "fused", "nfused", "x2", "prm2", "acc2")

    def __init__(self, x, bits, prm, mode, act, slope, acc, x2=None, prm2=None, acc2=None):
        self.x, self.bits, self.prm, self.mode, self.act, self.slope, self.acc = x, bits, prm, mode, act, slope, acc
        self.x2, self.prm2, self.acc2 = (x2, prm2, acc2) if mode == 3 and x2 is not None else (None, None, None)
        self.fused = None
        self.nfused = 0

    def mark_fused(self, g):
        self.fused = (g.data_ptr(), g._version, tuple(g.shape), g.stride())
        self.nfused += 1

    def take(self, dout):
        """True when ``acc`` already holds the reduction of exactly ``dout``."""
        if self.fused is None:
            return False
        ok = self.nfused == 1 and self.fused == (dout.data_ptr(), dout._version, tuple(dout.shape), dout.stride())
        if not ok:
            self.acc.zero_()  # partial / foreign sums
            if self.acc2 is not None:
                self.acc2.zero_()
        self.fused = None
        self.nfused = 0
        return ok


def _nrows(x):
    N, C, H, W = x.shape
    return N * H * W


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, stats, weight, bias, running_mean, running_var, residual, training, momentum, eps, act,
                slope, ws_fwd, ws_bwd, join=None, refbox=None, r_stats=None, r_weight=None, r_bias=None, r_rm=None,
                r_rv=None, r_cfg=None, xjoin=None, prod_bias=None, post_res=False, colsum=None, tickets=None):
        # xjoin (conv.GradJoin): another consumer of ``x`` stashes its gradient there (e.g. the
        # identity path of a pre-activation block); the backward apply pass adds it in place
        # r_*: a second, training-mode BatchNorm applied to ``residual`` inside the same pass
        # (a residual block's projection BN): out = act(bn(x) + bn_r(residual)); bn_r's output is
        # never materialised and its backward reads (dout, mask bits, residual) directly
        N, C, H, W = x.shape
        if ld_of(x) != C:
            raise NotImplementedError("BatchNorm on a padded channel view")
        dev = x.device
        st = stream_handle()
        L = lib()
        prm = torch.empty((4, C), dtype=F32, device=dev)  # scale, shift, mean, invstd
        scale, shift, mean, invstd = prm[0], prm[1], prm[2], prm[3]
        rows = N * H * W
        g = weight.detach() if weight is not None else None
        b = bias.detach() if bias is not None else None
        # small BatchNorm: the shard fold runs inside the apply pass (csrc/bn.hip "Small BatchNorms")
        # eager only: it removes two launches per BatchNorm from the host's issue path (Hourglass eager
        # +3 %); inside a captured graph the launches cost nothing on the host and the two-kernel form
        # measured 1.4 % faster (profiles/bn_fin_ab.txt). Both forms leave the shards zeroed.
        fin = (training and tickets is not None and r_cfg is None and FUSE_FINALIZE and L.bn_fin_ok(x.numel(), C)
               and not torch.cuda.is_current_stream_capturing())
        if training:
            if stats is None:
                stats = ws_fwd
                L.bn_stats(ptr(x), rows, C, ptr(stats), st)
            if not fin:
                L.bn_finalize(ptr(stats), C, float(rows), float(eps), float(momentum), ptr(g), ptr(b),
                              ptr(running_mean), ptr(running_var), ptr(mean), ptr(invstd), ptr(scale), ptr(shift), st)
        else:
            L.bn_eval_prep(C, float(eps), ptr(g), ptr(b), ptr(running_mean), ptr(running_var), ptr(scale), ptr(shift), st)
            if weight is not None and weight.requires_grad:  # dgamma needs xhat of the running stats
                mean.copy_(running_mean)
                torch.rsqrt(running_var + eps, out=invstd)
        rprm = None
        if r_cfg is not None:
            r_mom, r_eps, r_ws_fwd, r_ws_bwd = r_cfg
            rprm = torch.empty((4, C), dtype=F32, device=dev)
            L.bn_finalize(ptr(r_stats), C, float(rows), float(r_eps), float(r_mom), ptr(r_weight.detach()),
                          ptr(r_bias.detach()), ptr(r_rm), ptr(r_rv), ptr(rprm[2]), ptr(rprm[3]), ptr(rprm[0]),
                          ptr(rprm[1]), st)
        out = torch.empty_like(x)
        # activation mask in backward: recomputed from x (z = x*scale + shift) when there is no
        # residual; with a residual it is stored as bits by this pass (training, C % 8 == 0) or,
        # failing that, read back from the saved output. post_res: out = act(z) + residual (the
        # residual after the activation): the mask is z's, from x, and d residual = d out
        post = bool(post_res) and residual is not None and r_cfg is None
        bits = training and bool(act) and residual is not None and C % 8 == 0 and not post
        mask = torch.empty(x.numel() // 8, dtype=torch.uint8, device=dev) if bits else None
        rsc, rsh = (rprm[0], rprm[1]) if rprm is not None else (None, None)

        if fin:
            COUNTERS["bn_fin_fused"] += 1
            L.bn_fin_apply(ptr(stats), float(rows), float(eps), float(momentum), ptr(g), ptr(b), ptr(running_mean),
                           ptr(running_var), ptr(prm), ptr(tickets[0]), ptr(x), ptr(residual), ptr(out), x.numel(), C,
                           act, float(slope), ptr(mask), int(post), st)
        else:
            L.bn_apply(ptr(x), ptr(residual), ptr(out), x.numel(), C, ptr(scale), ptr(shift), act, float(slope),
                       ptr(mask), st, rscale=ptr(rsc) if rsc is not None else 0,
                       rshift=ptr(rsh) if rsh is not None else 0, post=int(post))
        keep_out = bool(act) and residual is not None and not bits and not post
        ctx.save_for_backward(x, mask if bits else (out if keep_out else None), weight, bias, prm,
                              residual if rprm is not None else None, rprm, r_weight, r_bias)
        ctx.r_ws_bwd = r_cfg[3] if r_cfg is not None else None
        ctx.bits = bits
        ctx.post = post
        ctx.cfg = (training, act, slope, residual is not None and not post)
        ctx.ws_bwd = ws_bwd
        ctx.join = join
        ctx.xjoin = xjoin
        ctx.colsum = colsum if (training and C % 8 == 0 and C <= 2048) else None
        ctx.has_prod_bias = prod_bias is not None
        ctx.prod_bias_param = prod_bias  # leaf parameter (not saved): its gradient may sink in place
        ctx.bnref = None
        ctx.tickets = tickets if fin else None
        if refbox is not None and training and ws_bwd is not None and C % 8 == 0 and (not act or bits or residual is None
                                                                                       or post):
            mode = 3 if bits else (2 if act else 1)
            dual = (residual, rprm, r_cfg[3]) if (rprm is not None and DUAL_BWD) else (None, None, None)
            ctx.bnref = BNRef(x, mask if bits else None, prm, mode, act, slope, ws_bwd, *dual)
            refbox.append(ctx.bnref)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, out, weight, bias, prm, r_x, rprm, r_weight, r_bias = ctx.saved_tensors
        training, act, slope, has_res = ctx.cfg
        scale, shift, mean, invstd = prm[0], prm[1], prm[2], prm[3]
        N, C, H, W = x.shape
        fused = ctx.bnref is not None and ctx.bnref.take(dout)
        fused2 = fused and ctx.bnref.x2 is not None  # the folded projection BN's sums came along
        dout = grad_nhwc(dout)
        if ld_of(dout) != C:
            dout = dout.contiguous(memory_format=torch.channels_last)
        dev = x.device
        st = stream_handle()
        L = lib()
        xg, xg2 = ctx.xjoin.take2() if ctx.xjoin is not None else (None, None)
        pb_sink = pb_grad = None
        if xg is not None and not isinstance(xg, torch.Tensor):
            xg = xg.materialize()
        if xg2 is not None and not isinstance(xg2, torch.Tensor):
            xg2 = xg2.materialize()
        foldable = lambda t: (t is not None and training and t.dtype == BF16  # noqa: E731
                              and tuple(t.shape) == tuple(x.shape) and t.is_contiguous(memory_format=torch.channels_last))
        # the other consumers' gradients are summed inside the apply pass, written over the first's buffer
        fold_x = foldable(xg)
        fold_x2 = fold_x and foldable(xg2)
        if xg2 is not None and not fold_x2:
            xg = xg2 if xg is None else xg + xg2
            fold_x = foldable(xg)
        COUNTERS["bwd_apply_two_addends"] += int(fold_x2)
        dx = xg if fold_x else torch.empty_like(x)
        # identity shortcut of a residual block: hand the shortcut consumer's dgrad the raw dout +
        # mask bits instead of writing dres = act'(z)*dout (csrc/conv_fwd.hip resbits epilogue)
        lazy = (LAZY_SHORTCUT and training and has_res and ctx.needs_input_grad[6] and ctx.bits and ctx.join is not None
                and ctx.join.can_stash() and dout.is_contiguous(memory_format=torch.channels_last) and rprm is None)
        dres = (torch.empty_like(x) if (has_res and ctx.needs_input_grad[6] and not lazy and rprm is None)
                else None)
        dgamma = dbeta = None
        want_affine = weight is not None and (ctx.needs_input_grad[2] or ctx.needs_input_grad[3])
        direct = False
        # small BatchNorm: the backward fold runs inside the apply pass (no bn_bwd_finalize launch)
        bfin = (ctx.tickets is not None and training and rprm is None and L.bn_fin_ok(x.numel(), C))
        if training or want_affine:
            # sum dz and sum dz*xhat (xhat from the batch statistics, or the running ones in eval)
            rows = N * H * W
            acc = ctx.ws_bwd if ctx.ws_bwd is not None else torch.zeros((STAT_SHARDS, 2, C), dtype=F32, device=dev)
            COUNTERS["bwd_reduce_fused" if fused else "bwd_reduce_pass"] += 1
            if not fused:  # else the producing dgrad's epilogue already reduced into acc
                L.bn_bwd_reduce(ptr(dout), ptr(out), ptr(x), rows, C, ptr(mean), ptr(invstd), ptr(scale), ptr(shift),
                                act, float(slope), ptr(acc), int(ctx.bits), st)
            sg = grad_sink(weight) if ctx.needs_input_grad[2] else None
            sb = grad_sink(bias) if ctx.needs_input_grad[3] else None
            direct = sg is not None and sb is not None
            if weight is not None and not direct:
                dgamma = torch.empty(C, dtype=F32, device=dev)
                dbeta = torch.empty(C, dtype=F32, device=dev)
            coef = torch.empty((3, C), dtype=F32, device=dev)
            # the producing conv's bias gradient = sum of this BN's input gradient, from the same sums
            # in the finalize (training statistics, no other gradient folded into dx)
            if ctx.has_prod_bias and ctx.needs_input_grad[23]:
                if training and xg is None:
                    pb_sink = grad_sink(ctx.prod_bias_param)
                    if pb_sink is None:
                        pb_grad = torch.zeros(C, dtype=F32, device=dev)
            if not bfin:
                L.bn_bwd_finalize(ptr(acc), C, float(rows), ptr(weight.detach() if weight is not None else None),
                                  ptr(mean), ptr(invstd), ptr(sg if direct else dgamma), ptr(sb if direct else dbeta),
                                  int(direct), ptr(coef[0]), ptr(coef[1]), ptr(coef[2]), st,
                                  xsum=ptr(pb_sink if pb_sink is not None else pb_grad))
        # residual join with the projection BN folded in: both input gradients from one pass
        dual = (DUAL_BWD and training and rprm is not None and ctx.bits and not fold_x and ctx.needs_input_grad[6]
                and dout.is_contiguous(memory_format=torch.channels_last))
        # the producing conv's bias gradient from this pass (conv.ColsumBox): only when dx is all of
        # x's gradient this pass knows of (every joined gradient folded in)
        box = ctx.colsum if (training and not dual and (xg is None or fold_x) and (xg2 is None or fold_x2)
                             and not L.deterministic()) else None
        if training and not dual and bfin:
            COUNTERS["bn_bwd_fin_fused"] += 1
            L.bn_bwd_fin_apply(ptr(acc), float(N * H * W), ptr(weight.detach() if weight is not None else None),
                               ptr(mean), ptr(invstd), ptr(sg if direct else dgamma), ptr(sb if direct else dbeta),
                               int(direct), ptr(pb_sink if pb_sink is not None else pb_grad), ptr(ctx.tickets[1]),
                               ptr(dout), ptr(out), ptr(x), ptr(dx), ptr(dres), x.numel(), C, ptr(scale), ptr(shift),
                               act, float(slope), int(ctx.bits), ptr(xg) if fold_x else 0,
                               ptr(xg2) if fold_x2 else 0, ptr(box.acc) if box is not None else 0, st)
            if box is not None:
                box.pending, box.version = True, dx._version
                dx._dv_colsum = box
        elif training and not dual:
            L.bn_bwd_apply(ptr(dout), ptr(out), ptr(x), ptr(dx), ptr(dres), x.numel(), C, ptr(coef[0]), ptr(coef[1]),
                           ptr(coef[2]), ptr(scale), ptr(shift), act, float(slope), int(ctx.bits), st,
                           addend=ptr(xg) if fold_x else 0, addend2=ptr(xg2) if fold_x2 else 0,
                           colsum=ptr(box.acc) if box is not None else 0)
            if box is not None:
                box.pending, box.version = True, dx._version
                dx._dv_colsum = box
        elif not training:
            if act and out is None:  # eval backward needs the mask: rebuild the output
                out = torch.empty_like(x)
                L.bn_apply(ptr(x), 0, ptr(out), x.numel(), C, ptr(scale), ptr(shift), act, float(slope), 0, st)
            L.bn_bwd_eval(ptr(dout), ptr(out), ptr(dx), ptr(dres), x.numel(), C, ptr(scale), act, float(slope), st)
        r_dgamma = r_dbeta = None
        if dual:
            COUNTERS["dual_apply"] += 1
            COUNTERS["dual_fused"] += int(fused2)
            coef_r, r_dgamma, r_dbeta = _residual_bn_coef(ctx, dout, out, r_x, rprm, r_weight, r_bias, act, slope, fused2)
            dres = torch.empty_like(r_x)
            L.bn_bwd_apply_dual(ptr(dout), ptr(out), ptr(x), ptr(r_x), ptr(dx), ptr(dres), x.numel(), C, ptr(coef),
                                ptr(coef_r), act, float(slope), st)
        elif rprm is not None:
            dres, r_dgamma, r_dbeta = _residual_bn_backward(ctx, dout, out, r_x, rprm, r_weight, r_bias, act, slope,
                                                            fused2)
        if ctx.post and ctx.needs_input_grad[6]:
            dres = dout  # d(act(z) + r)/dr = 1: the incoming gradient itself, no pass
        if lazy:
            from .conv import MaskedGrad

            COUNTERS["shortcut_lazy"] += 1
            dres = ctx.join.produce(MaskedGrad(dout, out, act, slope))  # `out` holds the mask bits
        elif ctx.join is not None and dres is not None:
            dres = ctx.join.produce(dres)  # folded into the shortcut consumer's dgrad epilogue
        if xg is not None and not fold_x:
            dx = dx + xg
        if ctx.has_prod_bias and ctx.needs_input_grad[23] and pb_sink is None and pb_grad is None:
            # eval statistics / a folded second gradient: reduce the final dx explicitly
            from .conv import _channel_sum

            pb_grad = _channel_sum(dx if dx.shape[1] == C else dx.contiguous(memory_format=torch.channels_last))
        return (dx, None, dgamma, dbeta, None, None, dres, None, None, None, None, None, None, None, None, None,
                None, r_dgamma, r_dbeta, None, None, None, None, pb_grad, None, None, None)


def _residual_bn_coef(ctx, dout, bits, r_x, rprm, r_weight, r_bias, act, slope, fused):
    """Folded residual BatchNorm, backward statistics: dz = act'(z)*dout from the mask bits (never
    materialised) reduced against xhat_r -- unless the consumer dgrad's epilogue already did
    (``fused``) -- then dgamma_r / dbeta_r and the coefficients of d(r_x) = kA*dz + kB*r_x + kC."""
    L = lib()
    st = stream_handle()
    N, C, H, W = r_x.shape
    rows = N * H * W
    mbits = int(bits is not None and ctx.bits)
    acc = ctx.r_ws_bwd
    if not fused:
        L.bn_bwd_reduce(ptr(dout), ptr(bits), ptr(r_x), rows, C, ptr(rprm[2]), ptr(rprm[3]), 0, 0, act, float(slope),
                        ptr(acc), mbits, st)
    sg = grad_sink(r_weight) if ctx.needs_input_grad[17] else None
    sb = grad_sink(r_bias) if ctx.needs_input_grad[18] else None
    direct = sg is not None and sb is not None
    dgamma = dbeta = None
    if not direct:
        dgamma = torch.empty(C, dtype=F32, device=r_x.device)
        dbeta = torch.empty(C, dtype=F32, device=r_x.device)
    coef = torch.empty((3, C), dtype=F32, device=r_x.device)
    L.bn_bwd_finalize(ptr(acc), C, float(rows), ptr(r_weight.detach()), ptr(rprm[2]), ptr(rprm[3]),
                      ptr(sg if direct else dgamma), ptr(sb if direct else dbeta), int(direct), ptr(coef[0]), ptr(coef[1]),
                      ptr(coef[2]), st)
    return coef, dgamma, dbeta


def _residual_bn_backward(ctx, dout, bits, r_x, rprm, r_weight, r_bias, act, slope, fused=False):
    """Backward of the folded residual BatchNorm on its own: statistics (_residual_bn_coef), then
    d(r_x) = kA*dz + kB*r_x + kC in a separate apply pass."""
    L = lib()
    st = stream_handle()
    C = r_x.shape[1]
    mbits = int(bits is not None and ctx.bits)
    coef, dgamma, dbeta = _residual_bn_coef(ctx, dout, bits, r_x, rprm, r_weight, r_bias, act, slope, fused)
    dr = torch.empty_like(r_x)
    L.bn_bwd_apply(ptr(dout), ptr(bits), ptr(r_x), ptr(dr), 0, r_x.numel(), C, ptr(coef[0]), ptr(coef[1]), ptr(coef[2]),
                   0, 0, act, float(slope), mbits, st)
    return (dr if ctx.needs_input_grad[6] else None), dgamma, dbeta


class _BNActPoolFn(torch.autograd.Function):
    """Training-mode BatchNorm -> activation -> MaxPool2d as one forward pass and two backward
    passes (csrc/pool.hip bn_act_maxpool_*): the BN output is never materialised, its gradient
    never written. Forward reads x once and writes the pooled output + u8 window indices;
    backward = fused (maxpool gather -> act' -> BN reduction), bn_bwd_finalize, fused (gather ->
    act' -> dx = kA*dz + kB*x + kC). Values, indices and gradients equal the unfused
    bn_apply -> maxpool chain (the BN output's bf16 rounding is kept before the max)."""

    @staticmethod
    def forward(ctx, x, stats, weight, bias, running_mean, running_var, momentum, eps, act, slope, ws_fwd, ws_bwd,
                k, s, p, P, Q):
        N, C, H, W = x.shape
        dev = x.device
        st = stream_handle()
        L = lib()
        prm = torch.empty((4, C), dtype=F32, device=dev)  # scale, shift, mean, invstd
        g = weight.detach() if weight is not None else None
        b = bias.detach() if bias is not None else None
        if stats is None:
            stats = ws_fwd
            L.bn_stats(ptr(x), N * H * W, C, ptr(stats), st)
        L.bn_finalize(ptr(stats), C, float(N * H * W), float(eps), float(momentum), ptr(g), ptr(b), ptr(running_mean),
                      ptr(running_var), ptr(prm[2]), ptr(prm[3]), ptr(prm[0]), ptr(prm[1]), st)
        y = torch.empty((N, C, P, Q), dtype=BF16, device=dev, memory_format=torch.channels_last)
        idx = torch.empty((N, P, Q, C), dtype=torch.uint8, device=dev)
        r = L.bn_act_maxpool_fwd(ptr(x), ptr(y), ptr(idx), N, H, W, C, P, Q, k[0], k[1], s[0], s[1], p[0], p[1],
                                 ptr(prm[0]), ptr(prm[1]), act, float(slope), st)
        if r != 0:
            raise RuntimeError("bn_act_maxpool_fwd: shape not covered (check bn_act_maxpool_ok first)")
        ctx.save_for_backward(x, idx, weight, bias, prm)
        ctx.cfg = (act, slope, k, s, p, P, Q)
        ctx.ws_bwd = ws_bwd
        return y

    @staticmethod
    def backward(ctx, dy):
        x, idx, weight, bias, prm = ctx.saved_tensors
        act, slope, k, s, p, P, Q = ctx.cfg
        N, C, H, W = x.shape
        dev = x.device
        st = stream_handle()
        L = lib()
        dy = grad_nhwc(dy)
        if ld_of(dy) != C or not dy.is_contiguous(memory_format=torch.channels_last):
            dy = dy.contiguous(memory_format=torch.channels_last)
        geo = (N, H, W, C, P, Q, k[0], k[1], s[0], s[1], p[0], p[1])
        acc = ctx.ws_bwd
        L.bn_act_maxpool_bwd(ptr(dy), ptr(idx), ptr(x), 0, *geo, ptr(prm), 0, act, float(slope), ptr(acc), 0, st)
        sg = grad_sink(weight) if ctx.needs_input_grad[2] else None
        sb = grad_sink(bias) if ctx.needs_input_grad[3] else None
        dgamma = dbeta = None
        coef = torch.empty((3, C), dtype=F32, device=dev)
        direct = sg is not None and sb is not None
        if weight is not None and not direct:
            dgamma = torch.empty(C, dtype=F32, device=dev)
            dbeta = torch.empty(C, dtype=F32, device=dev)
        L.bn_bwd_finalize(ptr(acc), C, float(N * H * W), ptr(weight.detach() if weight is not None else None),
                          ptr(prm[2]), ptr(prm[3]), ptr(sg if direct else dgamma), ptr(sb if direct else dbeta),
                          int(direct), ptr(coef[0]), ptr(coef[1]), ptr(coef[2]), st)
        dx = torch.empty_like(x)
        L.bn_act_maxpool_bwd(ptr(dy), ptr(idx), ptr(x), ptr(dx), *geo, ptr(prm), ptr(coef), act, float(slope), ptr(acc),
                             1, st)
        return (dx, None, dgamma, dbeta) + (None,) * 13


def bn_act_maxpool_ok(x, bn, pool):
    """Whether BN(training) -> act -> ``pool`` (an nn.MaxPool2d) can run as one fused op."""
    k = pool.kernel_size if isinstance(pool.kernel_size, tuple) else (pool.kernel_size, pool.kernel_size)
    d = pool.dilation if isinstance(pool.dilation, tuple) else (pool.dilation, pool.dilation)
    C = x.shape[1]
    return (native(x) and bn.training and bn.track_running_stats and C % 8 == 0 and 256 % (C // 8) == 0
            and d == (1, 1) and not pool.return_indices and k[0] * k[1] <= 255 and torch.is_grad_enabled())


def batch_norm_act_maxpool(x, bn, act, slope, pool, stats=None):
    """maxpool(act(BN(x))) with a training-mode ``bn`` as one fused native op (see _BNActPoolFn)."""
    from .pool import _pair, pool_out

    k, s, p = _pair(pool.kernel_size), _pair(pool.stride if pool.stride is not None else pool.kernel_size), _pair(pool.padding)
    N, C, H, W = x.shape
    P = pool_out(H, k[0], s[0], p[0], pool.ceil_mode)
    Q = pool_out(W, k[1], s[1], p[1], pool.ceil_mode)
    if bn.num_batches_tracked is not None:
        _count_batch(bn)
    ws_fwd = workspace(bn, "bn_fwd", (STAT_ROWS, C), x.device)
    ws_bwd = workspace(bn, "bn_bwd", (STAT_SHARDS, 2, C), x.device)
    return _BNActPoolFn.apply(x, stats, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn_momentum(bn), bn.eps,
                              ACT_IDS[act], float(slope), ws_fwd, ws_bwd, k, s, p, P, Q)


def conv_bn_act_maxpool(x, conv, bn, act, pool, slope=0.0):
    """conv -> BN -> act -> MaxPool2d (the ResNet stem): BN statistics from the conv epilogue, then
    the fused BN/act/pool op when it applies, else the unfused chain."""
    from .conv import conv2d
    from .pool import max_pool2d

    if not native(x):
        return pool(_torch_bn_act(conv(x), bn, act, slope, None))
    want = bn.training and bn.track_running_stats and conv.out_channels % 8 == 0
    if not want:
        return max_pool2d(conv_bn_act(x, conv, bn, act, slope), pool.kernel_size, pool.stride, pool.padding, pool.ceil_mode)
    sbuf = workspace(bn, "bn_fwd", (STAT_ROWS, conv.out_channels), x.device)
    pad = conv.native_padding(x.shape[2], x.shape[3]) if hasattr(conv, "native_padding") else conv.padding
    y, stats = conv2d(x, conv.weight, conv.bias, conv.stride, pad, conv.dilation, conv.groups, want_stats=True,
                      stats_buf=sbuf)
    if y.shape[1] % 8 != 0 or ld_of(y) != y.shape[1] or not bn_act_maxpool_ok(y, bn, pool):
        if ld_of(y) != y.shape[1]:
            y = y.contiguous(memory_format=torch.channels_last)
            stats = None
        z = batch_norm_act(y, bn, act, slope, None, stats)
        return max_pool2d(z, pool.kernel_size, pool.stride, pool.padding, pool.ceil_mode)
    return batch_norm_act_maxpool(y, bn, act, slope, pool, stats)


def masked_grad(grad, bits, act, slope):
    """act'(z) * grad with the mask stored as bits (1 per element, dense NHWC): the materialised
    form of a MaskedGrad, via the BN backward apply pass with unit coefficients."""
    C = grad.shape[1]
    g = grad if grad.is_contiguous(memory_format=torch.channels_last) else grad.contiguous(memory_format=torch.channels_last)
    out = torch.empty_like(g)
    one = torch.ones(C, dtype=F32, device=g.device)
    zero = torch.zeros(C, dtype=F32, device=g.device)
    lib().bn_bwd_apply(ptr(g), ptr(bits), ptr(g), ptr(out), 0, g.numel(), C, ptr(one), ptr(zero), ptr(zero), ptr(one),
                       ptr(zero), act, float(slope), 1, stream_handle())
    return out


def _torch_bn_act(x, bn, act, slope, residual):
    y = bn(x) if bn is not None else x
    if residual is not None:
        y = y + residual
    if act == "relu":
        y = TF.relu(y)
    elif act in ("leaky", "leaky_relu"):
        y = TF.leaky_relu(y, slope)
    return y


def _flush_batch_count(bn):
    d = bn.__dict__
    n = d.get("_dv_nbt_pending", 0)
    if n:
        if not _nbt_rewritten(bn):
            bn.num_batches_tracked.add_(n)
        d["_dv_nbt_pending"] = 0


def _nbt_rewritten(bn) -> bool:
    """Was ``num_batches_tracked`` written in place since the pending count started
    (reset_running_stats' zero_, load_state_dict's copy_)? Those writes replace the count. A
    different tensor object (deepcopy, module.to / cuda) carries the count over."""
    t = bn.num_batches_tracked
    ref = bn.__dict__.get("_dv_nbt_ver")
    return ref is not None and ref[0] == id(t) and ref[1] != t._version


def _count_batch(bn):
    """``num_batches_tracked += 1`` with torch semantics, but counted on the host and written to
    the device buffer lazily (before any state_dict / when momentum=None needs it): one tiny
    kernel per BN layer per step otherwise (53 launches per ResNet-50 step)."""
    if bn.momentum is None:
        _flush_batch_count(bn)
        bn.num_batches_tracked.add_(1)
        return
    d = bn.__dict__  # plain instance attributes: no nn.Module.__setattr__ on the per-call path
    if "_dv_nbt_hook" not in d:
        d["_dv_nbt_hook"] = bn.register_state_dict_pre_hook(lambda m, *a, **k: _flush_batch_count(m))
    add_pending_batches(bn, 1)


def add_pending_batches(bn, k):
    """Count ``k`` more training batches against ``bn.num_batches_tracked`` (host side, lazy)."""
    d = bn.__dict__
    t = bn.num_batches_tracked
    if d.get("_dv_nbt_pending", 0) and _nbt_rewritten(bn):
        d["_dv_nbt_pending"] = 0  # the buffer was rewritten since: earlier pending steps are void
    d["_dv_nbt_pending"] = d.get("_dv_nbt_pending", 0) + k
    d["_dv_nbt_ver"] = (id(t), t._version)


def bn_momentum(bn) -> float:
    """Exponential-average factor with torch semantics (momentum=None -> cumulative)."""
    if bn.momentum is None:
        return 1.0 / float(bn.num_batches_tracked.item())
    return bn.momentum


def batch_norm_act(x, bn, act=None, slope=0.0, residual=None, stats=None, residual_join=None, residual_bn=None,
                   input_join=None, prod_bias=None, residual_post=False, colsum=None):
    """act(BN(x) (+ residual)) with ``bn`` an nn.BatchNorm2d (parameters, buffers, mode).
    ``input_join`` (conv.GradJoin): x's gradient from another consumer, stashed there by its
    producer, is added inside this BN's backward apply pass.
    ``colsum`` (conv.ColsumBox): x is a conv output with a bias; the backward apply pass sums x's
    gradient per channel for that bias (see conv2d bias_colsum).
    ``residual_bn=(bn_r, stats_r)``: ``residual`` is a raw conv output still to be normalised by
    ``bn_r`` (training mode, batch statistics ``stats_r`` from its conv epilogue); the two BNs,
    the add and the activation run as one pass (see conv_bn_deferred)."""
    if residual_bn is not None:
        rbn, rstats = residual_bn
        C = x.shape[1]
        fold = (native(x) and bn.training and rbn.training and rbn.track_running_stats and rstats is not None
                and rbn.affine and C % 8 == 0 and (act is None or act in ("relu", "leaky", "leaky_relu"))
                and is_nhwc(residual) and ld_of(residual) == C and ld_of(x) == C)
        if not fold:
            residual = batch_norm_act(residual, rbn, None, 0.0, None, rstats)
            residual_bn = None
    if not native(x):
        if residual_post and residual is not None:
            return _torch_bn_act(x, bn, act, slope, None) + residual
        return _torch_bn_act(x, bn, act, slope, residual)
    training = bn.training or not bn.track_running_stats
    if bn.training and bn.track_running_stats and bn.num_batches_tracked is not None:
        _count_batch(bn)
    mom = bn_momentum(bn) if bn.training and bn.track_running_stats else 0.0
    rm = bn.running_mean if bn.track_running_stats else None
    rv = bn.running_var if bn.track_running_stats else None
    if not (x.dtype == BF16 and is_nhwc(x) and ld_of(x) == x.shape[1]):
        x = x.to(dtype=BF16).contiguous(memory_format=torch.channels_last)
    if residual is not None and not (is_nhwc(residual) and ld_of(residual) == residual.shape[1]):
        residual = residual.to(dtype=BF16).contiguous(memory_format=torch.channels_last)
        residual_join = None  # the residual reaches its source through a copy
    C = x.shape[1]
    ws_fwd = workspace(bn, "bn_fwd", (STAT_ROWS, C), x.device) if training else None
    ws_bwd = workspace(bn, "bn_bwd", (STAT_SHARDS, 2, C), x.device) if training else None
    refbox = [] if FUSE_BWD_STATS and torch.is_grad_enabled() else None
    rargs = ()
    if residual_bn is not None:
        rbn, rstats = residual_bn
        if rbn.num_batches_tracked is not None:
            _count_batch(rbn)
        rargs = (rstats, rbn.weight, rbn.bias, rbn.running_mean, rbn.running_var,
                 (bn_momentum(rbn), rbn.eps, workspace(rbn, "bn_fwd", (STAT_ROWS, C), x.device),
                  workspace(rbn, "bn_bwd", (STAT_SHARDS, 2, C), x.device)))
    if not rargs:
        rargs = (None,) * 6
    y = _BN_APPLY(x, stats, bn.weight, bn.bias, rm, rv, residual, training, mom,
                       bn.eps, ACT_IDS[act], float(slope), ws_fwd, ws_bwd, residual_join, refbox, *rargs, input_join,
                       prod_bias, bool(residual_post and residual_bn is None), colsum,
                       workspace(bn, "bn_fin_ticket", (2, C // 64), x.device, torch.int32)
                       if training and C % 64 == 0 else None)
    if refbox:
        y._dv_bnref = refbox[0]  # read by the consumer conv (ops.conv._ConvFn)
    return y


def conv_bn_deferred(x, conv, bn, join=None, join_role=None):
    """conv -> BatchNorm whose apply pass is deferred into its consumer's BN pass (a residual
    block's projection shortcut, folded into the block's last BN+add+ReLU by
    ``conv_bn_act(..., residual=y, residual_bn=rbn)``). Returns ``(y, rbn)``: the raw conv output
    and ``(bn, stats)``, or the normal BN output and None when the fold does not apply."""
    from .conv import conv2d

    ok = (FOLD_RESIDUAL_BN and native(x) and bn.training and bn.track_running_stats and bn.affine
          and conv.out_channels % 8 == 0 and torch.is_grad_enabled())
    if not ok:
        return conv_bn_act(x, conv, bn, join=join, join_role=join_role), None
    sbuf = workspace(bn, "bn_fwd", (STAT_ROWS, conv.out_channels), x.device)
    pad = conv.native_padding(x.shape[2], x.shape[3]) if hasattr(conv, "native_padding") else conv.padding
    y, stats = conv2d(x, conv.weight, conv.bias, conv.stride, pad, conv.dilation, conv.groups, want_stats=True,
                      stats_buf=sbuf, join=join, join_role=join_role)
    return y, (bn, stats)


def conv_bn_act(x, conv, bn, act=None, slope=0.0, residual=None, join=None, join_role=None, residual_join=None,
                residual_bn=None, reflect_pad=None, shuffle=0, residual_post=False):
    """Fused conv -> BN (batch stats from the conv epilogue) -> (+residual) -> activation.

    ``shuffle=g``: conv -> channel shuffle (g groups) -> BN -> act, the shuffle fused into the
    grouped conv's store (csrc/gconv.hip; ShuffleNet V1).

    ``join`` / ``join_role`` ('consumer' | 'producer') and ``residual_join``: a conv.GradJoin
    shared by the two consumers of a block input (see models/resnet.py) so the gradient sum
    is folded into the consumer conv's dgrad epilogue."""
    from .conv import conv2d

    if not native(x):
        if residual_bn is not None:
            residual = _torch_bn_act(residual, residual_bn[0], None, 0.0, None)
        if reflect_pad is not None:
            p = (reflect_pad, reflect_pad) if isinstance(reflect_pad, int) else tuple(reflect_pad)
            x = TF.pad(x, (p[1], p[1], p[0], p[0]), mode="reflect")
        y = conv(x)
        if shuffle and shuffle > 1:
            from .concat import channel_shuffle

            y = channel_shuffle(y, shuffle)
        if residual_post and residual is not None:
            return _torch_bn_act(y, bn, act, slope, None) + residual
        return _torch_bn_act(y, bn, act, slope, residual)
    # BN kernels need dense channels: a channel count that is not a multiple of 8 comes back as a
    # padded view, which is compacted below and gets its statistics from a separate pass
    want = (bn.training or not bn.track_running_stats) and conv.out_channels % 8 == 0
    sbuf = workspace(bn, "bn_fwd", (STAT_ROWS, conv.out_channels), x.device) if want else None
    pad = conv.native_padding(x.shape[2], x.shape[3]) if hasattr(conv, "native_padding") else conv.padding
    mode = "zeros"
    if reflect_pad is not None:  # ReflectionPad2d in front of a pad-0 conv: fused into the gather
        pad, mode = reflect_pad, "reflect"
    bvb = conv.bias is not None and bn.training and not shuffle  # bias gradient from the BN (bn_bwd_finalize xsum)
    r = conv2d(x, conv.weight, conv.bias, conv.stride, pad, conv.dilation, conv.groups, want_stats=want,
               stats_buf=sbuf, join=join, join_role=join_role, pad_mode=mode, shuffle=shuffle, bias_via_bn=bvb)
    y, stats = r if want else (r, None)
    prod_bias = conv.bias if (bvb and getattr(y, "_dv_bias_via_bn", False)) else None
    if y.shape[1] % 8 != 0:  # padded view: BN kernels require dense channels
        y = y.contiguous(memory_format=torch.channels_last)
        stats = None
    return batch_norm_act(y, bn, act, slope, residual, stats, residual_join=residual_join, residual_bn=residual_bn,
                          prod_bias=prod_bias, residual_post=residual_post)


_BN_APPLY = fast_apply(_BNActFn)
