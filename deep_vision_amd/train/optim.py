"""Fused optimizers over one flat fp32 parameter buffer.

All parameters of a group live in a single contiguous fp32 buffer (the ``nn.Parameter``s become
views into it) and their ``.grad``s are views into a matching flat gradient buffer. One kernel
launch (csrc/loss_optim.hip) updates the whole model per step, and the data-parallel layer
all-reduces slices of the same flat gradient buffer in place (no bucket copies).

Update rules match torch.optim.SGD / Adam / RMSprop exactly (same state names, same
``state_dict`` format), as used by the reference configs (R/ResNet/pytorch/train.py:26-215:
SGD momentum .9 + wd, RMSprop for MobileNet; Adam for LeNet/YOLO/Hourglass/GANs).
On CPU the same classes run the identical math with torch ops.
"""
from __future__ import annotations

import math

import torch

from .._ext import lib, ptr, stream_handle


class _FlatOptimizer(torch.optim.Optimizer):
    STATE_NAMES: tuple = ()

    def __init__(self, params, defaults):
        super().__init__(params, defaults)
        self._flat = []  # per group: dict(param, grad, views, gviews, offsets, states)
        for group in self.param_groups:
            self._flat.append(self._flatten_group(group))

    # ---------------- flat storage ----------------
    @staticmethod
    def _shared_span(ps, sizes):
        """(shared, lo, hi) when every parameter of ``ps`` is a view into ONE existing flat
        buffer pair (parallel.flat.flatten_parameters / another optimizer) and together they tile
        the contiguous range [lo, hi) of it exactly; otherwise None."""
        shared = getattr(ps[0], "_dv_flat", None)
        if shared is None or any(getattr(p, "_dv_flat", None) is not shared for p in ps):
            return None
        spans = sorted((p._dv_off, n) for p, n in zip(ps, sizes))
        lo = spans[0][0]
        end = lo
        for off, n in spans:
            if off != end:
                return None
            end += n
        for p, n in zip(ps, sizes):  # each parameter must still BE its slice of the buffer
            if p.data_ptr() != shared[0][p._dv_off:p._dv_off + n].data_ptr():
                return None
        return shared, lo, end

    def _flatten_group(self, group, old=None):
        ps = group["params"]
        if not ps:
            return None
        dev = ps[0].device
        for p in ps:
            if p.dtype != torch.float32:
                raise TypeError("fused optimizers keep fp32 master parameters")
            if p.device != dev:
                raise ValueError("all parameters of a group must live on one device")
        # reuse an existing flat buffer (parallel.flat.flatten_parameters) when the group's
        # parameters are views that tile a contiguous range of it
        sizes = [p.numel() for p in ps]
        total = sum(sizes)
        span = self._shared_span(ps, sizes)
        views, gviews, offs = [], [], []
        if span is not None:
            shared, lo, hi = span
            pflat, gflat = shared[0][lo:hi], shared[1][lo:hi]
            for p, n in zip(ps, sizes):
                off = p._dv_off - lo
                views.append(pflat[off:off + n].view(p.shape))
                gviews.append(gflat[off:off + n].view(p.shape))
                if p.grad is not None and p.grad.data_ptr() != gviews[-1].data_ptr():
                    gviews[-1].copy_(p.grad)
                p.data = views[-1]
                p.grad = gviews[-1]
                offs.append((off, n))
        else:
            shared = None
            pflat = torch.empty(total, dtype=torch.float32, device=dev)
            gflat = torch.zeros(total, dtype=torch.float32, device=dev)
            off = 0
            for p, n in zip(ps, sizes):
                pv = pflat[off:off + n].view(p.shape)
                gv = gflat[off:off + n].view(p.shape)
                pv.copy_(p.data)
                p.data = pv
                if p.grad is not None:
                    gv.copy_(p.grad)
                p.grad = gv
                views.append(pv)
                gviews.append(gv)
                offs.append((off, n))
                off += n
            shared = (pflat, gflat)
            for p in ps:
                p._dv_flat = shared
            for p, (off, _) in zip(ps, offs):
                p._dv_off = off
        states = {name: torch.zeros(total, dtype=torch.float32, device=dev) for name in self.STATE_NAMES}
        f = dict(param=pflat, grad=gflat, views=views, gviews=gviews, offsets=offs, states=states, step=0,
                 first=True, shared=shared)
        if old is not None:  # re-bound after the parameters moved: carry the optimizer state over
            f["step"], f["first"] = old["step"], old["first"]
            if old.get("hp") is not None:
                f["hp"] = old["hp"]
            for (o_off, n), (n_off, _) in zip(old["offsets"], offs):
                for name in self.STATE_NAMES:
                    f["states"][name][n_off:n_off + n].copy_(old["states"][name][o_off:o_off + n])
        return f

    def _check_binding(self):
        """Each parameter must still be a view of THIS optimizer's flat buffer. When a later
        ``parallel.DataParallel`` (or anything calling flatten_parameters) moved the parameters
        into a new flat buffer, re-bind transparently -- updating the orphaned old buffer would
        leave the model untrained -- and carry the state over."""
        for gi, (group, f) in enumerate(zip(self.param_groups, self._flat)):
            if f is None:
                continue
            shared = f["shared"]
            if all(getattr(p, "_dv_flat", None) is shared and p.data_ptr() == v.data_ptr()
                   for p, v in zip(group["params"], f["views"])):
                continue
            if f["param"].is_cuda and torch.cuda.is_current_stream_capturing():
                raise RuntimeError("parameters were re-flattened under a graph capture")
            self._flat[gi] = self._flatten_group(group, old=f)
            self._rebinds = getattr(self, "_rebinds", 0) + 1

    # ---------------- device-side hyperparameters (HIP-graph replay) ----------------
    def use_device_hparams(self, on: bool = True):
        """Kernels read (lr, bias corrections) from a per-group device tensor ``hp`` instead of
        launch arguments, so a step captured in a HIP graph (train.graph.CapturedStep) follows LR
        schedules and Adam's step count: ``graph_tick()`` writes the next step's values before
        each replay.

        The tensor is allocated ONCE per group and never replaced: every captured graph bakes its
        device pointer in, so a second capture (another input signature) must share it -- a
        fresh tensor would leave the first graph reading freed memory."""
        for f in self._flat:
            if f is None:
                continue
            if on:
                if f.get("hp") is None:
                    f["hp"] = f.get("_hp_keep")
                if f["hp"] is None:
                    f["hp"] = torch.zeros(4, dtype=torch.float32, device=f["param"].device)
                f["_hp_keep"] = f["hp"]
            else:
                f["hp"] = None  # eager launches take host arguments; the buffer stays alive in _hp_keep

    def _hparams(self, group, step):
        """(lr, bias-correction-1, bias-correction-2) of step number ``step`` (1-based)."""
        return float(group["lr"]), 1.0, 1.0

    def _write_hp(self, group, f):
        lr, bc1, bc2 = self._hparams(group, f["step"])
        f["hp"].copy_(torch.tensor([lr, bc1, bc2, float(f["step"])], dtype=torch.float32))

    @torch.no_grad()
    def graph_tick(self):
        """Advance the host step counters as one eager step() would, and write the device
        hyperparameters of that step (ordered on the current stream before the replay)."""
        for group, f in zip(self.param_groups, self._flat):
            if f is None:
                continue
            f["step"] += 1
            f["first"] = False
            self._write_hp(group, f)

    def _hp_ptr(self, f):
        hp = f.get("hp")
        return 0 if hp is None else ptr(hp)

    # ---------------- device-side non-finite guard (HIP-graph replay) ----------------
    def use_device_guard(self, on: bool = True):
        """Skip-step on non-finite gradients decided ON THE DEVICE (csrc/loss_optim.hip
        nonfinite_check / nonfinite_tally): every step checks the flat gradients, the update
        kernels become no-ops when any is Inf/NaN, and device counters record the skips -- no host
        synchronisation, so it works inside a captured step. The guard
        tensor [flag, skipped, consecutive, last, applied] is allocated once and never replaced
        (graphs bake its pointer in). In a data-parallel step the checked gradients are the
        all-reduced ones, identical on every rank: the ranks skip together without an extra
        collective.

        ``applied`` counts the steps actually taken (it starts at the host step count): Adam's
        bias corrections read it under the guard, so a skipped replay does not advance them -- as
        an eager skipped step, which never calls step(), does not. The host step count
        (graph_tick, state_dict) and LR schedules still count every replay; the applied count is
        ``step - skipped``."""
        self._dguard_on = bool(on)
        if on and getattr(self, "_dguard", None) is None:
            dev = next((f["param"].device for f in self._flat if f is not None), None)
            if dev is not None and dev.type == "cuda":
                done = getattr(self, "_loaded_applied", None)
                if done is None:
                    done = max((f["step"] for f in self._flat if f is not None), default=0)
                self._dguard = torch.tensor([0.0, 0.0, 0.0, 0.0, float(done)], dtype=torch.float32, device=dev)

    def _guard_active(self):
        return getattr(self, "_dguard_on", False) and getattr(self, "_dguard", None) is not None

    def _skip_ptr(self):
        return ptr(self._dguard) if self._guard_active() else 0

    def device_guard_counts(self):
        """(steps skipped so far, current run of consecutive skips, last step skipped) -- one
        device->host read; call at the logging cadence."""
        if getattr(self, "_dguard", None) is None:
            return 0, 0, False
        v = self._dguard.tolist()
        return int(v[1]), int(v[2]), bool(v[3])

    def param_views(self):
        return [v for f in self._flat if f for v in f["views"]]

    def flat_grads(self):
        return [f["grad"] for f in self._flat if f]

    @torch.no_grad()
    def zero_grad(self, set_to_none: bool = False):
        self._check_binding()
        for group, f in zip(self.param_groups, self._flat):
            if f is None:
                continue
            f["grad"].zero_()
            for p, gv in zip(group["params"], f["gviews"]):
                if p.grad is not gv:
                    p.grad = gv

    def _sync_grads(self, group, f):
        """Ensure every .grad is the flat view; returns active (offset, n) segments."""
        segs = []
        all_active = True
        for p, gv, (off, n) in zip(group["params"], f["gviews"], f["offsets"]):
            g = p.grad
            if g is None:
                all_active = False
                p.grad = gv
                gv.zero_()
                continue
            if g is not gv:
                gv.copy_(g)
                p.grad = gv
            segs.append((off, n))
        if all_active:
            return [(0, f["param"].numel())]
        # merge adjacent segments
        merged = []
        for off, n in sorted(segs):
            if merged and merged[-1][0] + merged[-1][1] == off:
                merged[-1] = (merged[-1][0], merged[-1][1] + n)
            else:
                merged.append((off, n))
        return merged

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = 1.0):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._check_binding()
        guard = self._guard_active()
        # the active segments of every group, taken once: _sync_grads binds a None .grad to its
        # (zeroed) flat view, so a second call would report every parameter active and the update
        # would apply weight decay / momentum to parameters that got no gradient this step
        segs_all = [self._sync_grads(group, f) if f is not None else None
                    for group, f in zip(self.param_groups, self._flat)]
        if guard:  # flag any non-finite gradient of any group before the first update launch
            for f in self._flat:
                if f is not None:
                    lib().nonfinite_check(ptr(f["grad"]), f["grad"].numel(), ptr(self._dguard), stream_handle())
        for group, f, segs in zip(self.param_groups, self._flat, segs_all):
            if f is None:
                continue
            f["step"] += 1
            # device hyperparameters: an eager step writes its own; inside a graph capture the
            # values come from graph_tick() before each replay (a captured copy would replay stale)
            if f.get("hp") is not None and not torch.cuda.is_current_stream_capturing():
                self._write_hp(group, f)
            for off, n in segs:
                self._update(group, f, off, n, grad_scale)
            f["first"] = False
        if guard:
            lib().nonfinite_tally(ptr(self._dguard), stream_handle())  # counters; re-arms the flag
        if any(f is not None and f["param"].is_cuda for f in self._flat):
            from ..ops import wcache

            wcache.after_step()  # one batched re-layout of every cached bf16 weight operand
        return loss

    def _update(self, group, f, off, n, gs):  # pragma: no cover - abstract
        raise NotImplementedError

    @staticmethod
    def _slice(t, off, n):
        return t[off:off + n]

    # ---------------- torch-compatible state_dict ----------------
    def state_dict(self):
        sd = super().state_dict()
        state = {}
        idx = 0
        for group, f in zip(self.param_groups, self._flat):
            if f is None:
                continue
            for (off, n), p in zip(f["offsets"], group["params"]):
                st = {}
                for name, buf in f["states"].items():
                    st[name] = buf[off:off + n].view(p.shape).clone()
                if self.STATE_NAMES and not f["first"]:
                    st["step"] = torch.tensor(float(f["step"]))
                    state[idx] = st
                idx += 1
        sd["state"] = state
        # the device guard's applied-step count (steps whose update ran; Adam's bias corrections
        # follow it) and skips: a captured run's "step" also counts skipped replays, an eager run's
        # does not, so the applied count is saved explicitly
        applied = skipped = None
        if getattr(self, "_dguard", None) is not None:
            v = self._dguard.tolist()
            skipped, applied = int(v[1]), int(v[4])
        for g, f in zip(sd["param_groups"], self._flat):
            g["_dv_step"] = f["step"] if f else 0
            if applied is not None:
                g["_dv_applied"], g["_dv_skipped"] = applied, skipped
        return sd

    def load_state_dict(self, state_dict):
        groups = state_dict["param_groups"]
        for g, sg in zip(self.param_groups, groups):
            for k, v in sg.items():
                if k not in ("params", "_dv_step", "_dv_applied", "_dv_skipped"):
                    g[k] = v
        idx = 0
        for sg, group, f in zip(groups, self.param_groups, self._flat):
            if f is None:
                continue
            f["step"] = int(sg.get("_dv_step", 0))
            any_state = False
            for (off, n), p in zip(f["offsets"], group["params"]):
                st = state_dict["state"].get(idx, state_dict["state"].get(str(idx)))
                if st:
                    any_state = True
                    for name in self.STATE_NAMES:
                        if name in st:
                            f["states"][name][off:off + n].copy_(st[name].reshape(-1).to(f["param"].device))
                    if "step" in st and f["step"] == 0:
                        f["step"] = int(float(st["step"]))
                idx += 1
            f["first"] = not any_state
        # the device guard's applied-step count: saved by a guarded run, else every saved step applied
        saved = [sg["_dv_applied"] for sg in groups if "_dv_applied" in sg]
        self._loaded_applied = (int(saved[0]) if saved else
                                max((f["step"] for f in self._flat if f is not None), default=0))
        if getattr(self, "_dguard", None) is not None:
            self._dguard[4] = float(self._loaded_applied)


class FusedSGD(_FlatOptimizer):
    STATE_NAMES = ("momentum_buffer",)

    def __init__(self, params, lr=0.1, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False):
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                                      nesterov=nesterov))

    def _update(self, g, f, off, n, gs):
        p = f["param"][off:off + n]
        gr = f["grad"][off:off + n]
        buf = f["states"]["momentum_buffer"][off:off + n]
        if p.is_cuda:
            lib().sgd(ptr(p), ptr(gr), ptr(buf), n, float(g["lr"]), float(g["momentum"]), float(g["dampening"]),
                      float(g["weight_decay"]), int(g["nesterov"]), int(f["first"]), float(gs), stream_handle(),
                      hp=self._hp_ptr(f), skip=self._skip_ptr())
            return
        d = gr * gs + g["weight_decay"] * p
        if g["momentum"] != 0:
            if f["first"]:
                buf.copy_(d)
            else:
                buf.mul_(g["momentum"]).add_(d, alpha=1 - g["dampening"])
            d = d + g["momentum"] * buf if g["nesterov"] else buf
        p.add_(d, alpha=-g["lr"])


class FusedAdam(_FlatOptimizer):
    STATE_NAMES = ("exp_avg", "exp_avg_sq")

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, decoupled=False):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, decoupled=decoupled))

    def _hparams(self, group, step):
        b1, b2 = group["betas"]
        return float(group["lr"]), 1 - b1 ** step, 1 - b2 ** step

    def _update(self, g, f, off, n, gs):
        b1, b2 = g["betas"]
        _, bc1, bc2 = self._hparams(g, f["step"])
        p = f["param"][off:off + n]
        gr = f["grad"][off:off + n]
        m = f["states"]["exp_avg"][off:off + n]
        v = f["states"]["exp_avg_sq"][off:off + n]
        if p.is_cuda:
            lib().adam(ptr(p), ptr(gr), ptr(m), ptr(v), n, float(g["lr"]), float(b1), float(b2), float(g["eps"]),
                       float(g["weight_decay"]), int(g["decoupled"]), float(bc1), float(bc2), float(gs), stream_handle(),
                       hp=self._hp_ptr(f), skip=self._skip_ptr())
            return
        grad = gr * gs
        if g["decoupled"]:
            p.mul_(1 - g["lr"] * g["weight_decay"])
        else:
            grad = grad + g["weight_decay"] * p
        m.mul_(b1).add_(grad, alpha=1 - b1)
        v.mul_(b2).addcmul_(grad, grad, value=1 - b2)
        denom = (v / bc2).sqrt_().add_(g["eps"])
        p.addcdiv_(m, denom, value=-g["lr"] / bc1)


class FusedRMSprop(_FlatOptimizer):
    STATE_NAMES = ("square_avg", "momentum_buffer", "grad_avg")

    def __init__(self, params, lr=1e-2, alpha=0.99, eps=1e-8, weight_decay=0.0, momentum=0.0, centered=False):
        super().__init__(params, dict(lr=lr, alpha=alpha, eps=eps, weight_decay=weight_decay, momentum=momentum,
                                      centered=centered))

    def _update(self, g, f, off, n, gs):
        p = f["param"][off:off + n]
        gr = f["grad"][off:off + n]
        sq = f["states"]["square_avg"][off:off + n]
        mom = f["states"]["momentum_buffer"][off:off + n]
        ga = f["states"]["grad_avg"][off:off + n]
        if p.is_cuda:
            lib().rmsprop(ptr(p), ptr(gr), ptr(sq), ptr(mom), ptr(ga), n, float(g["lr"]), float(g["alpha"]),
                          float(g["eps"]), float(g["weight_decay"]), float(g["momentum"]), int(g["centered"]), float(gs),
                          stream_handle(), hp=self._hp_ptr(f), skip=self._skip_ptr())
            return
        grad = gr * gs + g["weight_decay"] * p
        sq.mul_(g["alpha"]).addcmul_(grad, grad, value=1 - g["alpha"])
        if g["centered"]:
            ga.mul_(g["alpha"]).add_(grad, alpha=1 - g["alpha"])
            avg = (sq - ga * ga).sqrt_().add_(g["eps"])
        else:
            avg = sq.sqrt().add_(g["eps"])
        if g["momentum"] > 0:
            mom.mul_(g["momentum"]).addcdiv_(grad, avg)
            p.add_(mom, alpha=-g["lr"])
        else:
            p.addcdiv_(grad, avg, value=-g["lr"])


OPTIMIZERS = {"SGD": FusedSGD, "Adam": FusedAdam, "RMSprop": FusedRMSprop}
