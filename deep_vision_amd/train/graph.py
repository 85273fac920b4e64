"""One training step captured as a HIP graph and replayed (``torch.cuda.CUDAGraph`` is hipGraph on
ROCm): the host launches the whole step -- forward, loss, backward, fused optimizer update and the
batched bf16 weight re-layout -- as one graph launch instead of one launch per kernel.

Where it pays: models whose step is launch-bound. The Stacked Hourglass step issues ~3,000 kernels
(4 stacks x 4 recursion levels of residual blocks on 4x4 - 64x64 maps, many of them a few
microseconds long); YOLOv3 ~800. A GPU-bound step (ResNet-50 at batch 256: 14.8 ms of host
enqueue under 21.7 ms of kernels, tools/graph_step.py) gains nothing.

What a replay does and does not redo:
  * every kernel of the captured step runs, on the same static buffers: inputs are copied into
    ``static_inputs`` before each replay (``__call__``), outputs are the static tensors returned by
    the captured call;
  * optimizer hyperparameters come from a device tensor the host writes before each replay
    (``_FlatOptimizer.use_device_hparams`` / ``graph_tick``): LR schedules and Adam's bias
    correction stay exact, and the host step counters advance as in eager mode;
  * BatchNorm ``num_batches_tracked`` is counted on the host per replay (running mean / var are
    updated on the device by the captured finalize kernels);
  * Python-side control flow is frozen at capture: shapes, the set of parameters that receive
    gradients and data-dependent branches must not change between steps.
Data parallel steps are captured too: the bucketed all-reduces that
parallel.DataParallel issues from autograd hooks during the capture are RCCL collectives on the
process group's stream, forked from and joined back to the capturing stream by events -- both
recorded into the graph -- so every replay re-runs the reductions in the captured bucket order,
overlapped with the captured backward exactly as in eager mode. Requirements: every rank captures
and replays the same step (lockstep), the communicator is initialised by the eager warm-up steps,
and ProcessGroupNCCL's async error handling is off (``TORCH_NCCL_ASYNC_ERROR_HANDLING=0``: its
watchdog cannot query events of a captured collective). ``DataParallel.comm_stats`` counts the
capture's issues only.
"""
from __future__ import annotations

from typing import Callable, Sequence

import torch


class CapturedStep:
    """``step_fn(*static_inputs)`` (zero_grad, forward, loss, backward, optimizer.step) captured once
    after ``warmup`` eager iterations on a side stream, then replayed by ``__call__``.

    >>> cap = CapturedStep(step, opt, (x_static, y_static), model=model)
    >>> loss = cap(x_batch, y_batch)        # copies into the static inputs, replays
    """

    def __init__(self, step_fn: Callable, optimizer, static_inputs: Sequence[torch.Tensor] = (), model=None,
                 warmup: int = 2):
        import os

        if torch.distributed.is_available() and torch.distributed.is_initialized() \
                and torch.distributed.get_backend() == "nccl" \
                and os.environ.get("TORCH_NCCL_ASYNC_ERROR_HANDLING", "") not in ("0",):
            raise RuntimeError("capturing RCCL collectives needs TORCH_NCCL_ASYNC_ERROR_HANDLING=0 set before the "
                               "process group is created (train.graph.prepare_capture_env)")
        if torch.distributed.is_available() and torch.distributed.is_initialized() \
                and torch.distributed.get_backend() == "gloo":
            raise RuntimeError("gloo collectives run on the host and cannot be captured in a HIP graph")
        if not hasattr(optimizer, "use_device_hparams"):
            raise TypeError("CapturedStep needs a fused optimizer (train.optim) with device hyperparameters")
        self.step_fn = step_fn
        self.opt = optimizer
        self.static_inputs = tuple(static_inputs)
        self._bns = []
        if model is not None:
            for m in model.modules():
                if isinstance(m, torch.nn.modules.batchnorm._BatchNorm) and m.track_running_stats:
                    if m.momentum is None:
                        raise RuntimeError("CapturedStep: BatchNorm(momentum=None) reads num_batches_tracked on "
                                           "the host every step and cannot be captured")
                    self._bns.append(m)
        self.graph = torch.cuda.CUDAGraph()
        self.outputs = None
        self.warmup_outputs = None  # what the last eager warm-up step returned (a real step)
        self._capture(warmup)

    def _capture(self, warmup):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s), capture_warmup():
            for _ in range(max(1, warmup)):  # real steps: allocator warm-up, first-step optimizer state
                self.warmup_outputs = self.step_fn(*self.static_inputs)
        torch.cuda.current_stream().wait_stream(s)
        from ..ops.act import step_counter

        step_counter(torch.cuda.current_device())  # exists before the capture (captured dropouts read it)
        torch.cuda.synchronize()
        self.opt.use_device_hparams(True)
        host = [(f["step"], f["first"]) if f else None for f in self.opt._flat]
        pending = {id(m): m.__dict__.get("_dv_nbt_pending", 0) for m in self._bns}
        # captured on the warm-up stream: the per-stream scratch the warm-up sized (split-K slabs,
        # channel sums) is what the captured kernels use -- a fresh capture stream would find none
        # and could not allocate it mid-capture
        from ..parallel.watchdog import suspend_polling

        with suspend_polling(), torch.cuda.graph(self.graph, stream=s):  # no event queries mid-capture
            self.outputs = self.step_fn(*self.static_inputs)
        # the capture executed nothing: undo its host-side bookkeeping
        for f, h in zip(self.opt._flat, host):
            if f is not None:
                f["step"], f["first"] = h
        self._counted = [m for m in self._bns if m.__dict__.get("_dv_nbt_pending", 0) != pending[id(m)]]
        for m in self._counted:
            m._dv_nbt_pending = pending[id(m)]

    def __call__(self, *inputs):
        for dst, src in zip(self.static_inputs, inputs):
            if src is not dst:
                dst.copy_(src, non_blocking=True)
        self.opt.graph_tick()
        from ..ops.bn import add_pending_batches

        for m in self._counted:
            add_pending_batches(m, 1)
        from ..ops.act import advance_dropout_step

        advance_dropout_step()  # fresh dropout masks per replay (ops/act.py)
        self.graph.replay()
        return self.outputs


_WARMUP = [0]


class capture_warmup:
    """Context of the eager steps that precede a capture: code that behaves differently under
    capture (models/hourglass.py branch streams) takes its capture-time form here too, so the
    warm-up sizes the same per-stream scratch the captured step will use."""

    def __enter__(self):
        _WARMUP[0] += 1
        return self

    def __exit__(self, *exc):
        _WARMUP[0] -= 1
        return False


def capturing_or_warming() -> bool:
    return _WARMUP[0] > 0 or torch.cuda.is_current_stream_capturing()


def prepare_capture_env() -> None:
    """Call before the process group is created when steps will be captured (see module doc)."""
    import os

    os.environ["TORCH_NCCL_ASYNC_ERROR_HANDLING"] = "0"


class GraphedTrainStep:
    """Trainer-side wrapper (train.engine.Engine.train_step): ``forward_loss(*inputs) -> (loss,
    extra)`` plus backward and optimizer step, captured on the first batch of each new input
    signature (shapes / dtypes of the flattened inputs) and replayed for every later batch with
    that signature. The capturing call trains on its own batch (the eager warm-up step). Up to
    ``max_graphs`` signatures are captured (default 2: the full batch and a short last batch of
    an epoch each get a graph and a private memory pool); further signatures run eagerly through
    ``eager_step``. All graphs of one optimizer share its single device hyperparameter tensor
    (``_FlatOptimizer.use_device_hparams`` never re-allocates it), so ``graph_tick`` before a
    replay reaches whichever graph runs."""

    def __init__(self, model, optimizer, forward_loss: Callable, eager_step: Callable, max_graphs: int = 2):
        self.model, self.opt, self.forward_loss, self.eager_step = model, optimizer, forward_loss, eager_step
        self.max_graphs = max_graphs
        from ..parallel.ddp import DataParallel

        self.ddp = model if isinstance(model, DataParallel) else None
        self.graphs = {}  # signature -> (CapturedStep, treespec)

    @staticmethod
    def _signature(flat):
        return tuple((tuple(t.shape), t.dtype, t.device) if isinstance(t, torch.Tensor) else ("const", t) for t in flat)

    def __call__(self, *inputs):
        from torch.utils._pytree import tree_flatten, tree_unflatten

        flat, spec = tree_flatten(inputs)
        if not all(isinstance(t, torch.Tensor) and t.is_cuda for t in flat):
            return self.eager_step(*inputs)
        sig = self._signature(flat)
        entry = self.graphs.get(sig)
        if entry is not None:
            return entry[0](*flat)
        if len(self.graphs) >= self.max_graphs:
            return self.eager_step(*inputs)
        static = [t.detach().clone() for t in flat]
        fl, opt, ddp = self.forward_loss, self.opt, self.ddp

        def step_fn(*st):
            args = tree_unflatten(list(st), spec)
            opt.zero_grad()
            loss, extra = fl(*args)
            loss.backward()
            if ddp is not None:
                ddp.finish()  # joins the bucket all-reduces back into the (captured) stream
            opt.step(grad_scale=ddp.grad_scale if ddp is not None else 1.0)
            return loss, extra

        cap = CapturedStep(step_fn, opt, static, model=ddp.module if ddp is not None else self.model, warmup=1)
        self.graphs[sig] = (cap, spec)
        return cap.warmup_outputs
