"""Shared training runtime of every family trainer (replaces DataParallel / MirroredStrategy glue).

``Engine`` owns: the process group (one rank per GPU, RCCL; gloo on CPU), the device, the model
(optionally wrapped in parallel.DataParallel -- bucketed RCCL all-reduce overlapped with
backward), the fused flat-buffer optimizer, the optimizer step with the 1/world averaging fused
in, the non-finite guard, the fault injector, the watchdog heartbeat and the step timer.

Loss scaling follows the reference per family: PT classifiers average over the *local* batch
(``nn.CrossEntropyLoss`` mean; DataParallel computed it over the global batch on GPU0, which
equals the mean of per-rank means for equal shards), TF2 loops sum per-example losses and
divide by the *global* batch (MirroredStrategy) -- ``Engine.world`` and
``TrainConfig.global_batch`` give both.
"""
from __future__ import annotations

import contextlib
import os
import random

import numpy as np
import torch

from .. import models as M
from ..parallel import dist as D
from ..parallel.ddp import DataParallel
from ..parallel.watchdog import CommWatchdog, install_backend_error_handling
from ..profiling import StepTimer
from ..utils.fault import FaultInjector, NonFiniteGuard, Watchdog
from .optim import FusedAdam, FusedRMSprop, FusedSGD

OPTIMIZERS = {"sgd": FusedSGD, "adam": FusedAdam, "rmsprop": FusedRMSprop}


def seed_everything(seed: int, rank: int = 0):
    random.seed(seed + rank)
    np.random.seed(seed + rank)
    torch.manual_seed(seed + rank)


def make_optimizer(name, params, kw):
    kw = dict(kw)
    if "betas" in kw:
        kw["betas"] = tuple(kw["betas"])
    return OPTIMIZERS[name](params, **kw)


class Engine:
    def __init__(self, device: str | None = None, backend: str | None = None, bucket_mb: float = 64.0,
                 log_every: int = 10, watchdog_s: float | None = None, profile: bool = False, graph: bool = False):
        if device == "cpu":
            backend = backend or "gloo"
        if graph:
            from .graph import prepare_capture_env

            prepare_capture_env()  # captured RCCL collectives: async error handling off (before init)
        install_backend_error_handling()  # RCCL async errors abort the communicator (before init)
        self.world, self.rank, self.local_rank, dev = D.init_distributed(backend)
        self.device = torch.device(device) if device and device != "cuda" else dev
        self.bucket_mb = bucket_mb
        self.is_main = self.rank == 0
        self.guard = NonFiniteGuard(every=log_every)
        self.faults = FaultInjector(rank=self.rank)
        self.timer = StepTimer(enabled=profile)
        wd = float(os.environ.get("DV_WATCHDOG_S", watchdog_s or 0))
        self.watchdog = Watchdog(wd).start() if wd > 0 else None
        # a hung / failed gradient all-reduce ends this rank with a non-zero exit (the launcher
        # then tears the job down) instead of blocking the whole job forever
        self.comm_watchdog = CommWatchdog().start() if self.world > 1 else None
        self.step_count = 0
        # HIP-graph replay of the whole step (train/graph.py), data-parallel all-reduces included.
        # In this mode the non-finite skip is decided on the device inside the captured step
        # (optimizer.use_device_guard), and every replay is tracked by the comm watchdog through an
        # event recorded after it (CommWatchdog.track). Host-side fault injection needs the eager step.
        self.graph = bool(graph) and self.device.type == "cuda"
        if graph and not self.graph:
            self.log("[dv] --graph needs a GPU: running eagerly")
        self._graphed = {}
        # eager steps run on a high-priority stream (as bench.py's): the weight-gradient side stream
        # then fills the CUs the main path leaves idle (profiles/main_stream_priority_ab.txt);
        # DV_MAIN_PRIO=0 keeps the default stream
        self.main_stream = None
        if self.device.type == "cuda" and not self.graph and os.environ.get("DV_MAIN_PRIO", "1") == "1":
            self.main_stream = torch.cuda.Stream(device=self.device, priority=-1)
            self.main_stream.wait_stream(torch.cuda.current_stream(self.device))
            torch.cuda.set_stream(self.main_stream)

    def log(self, *a, **kw):
        if self.is_main:
            print(*a, **kw, flush=True)

    # ---------------- model / optimizer ----------------
    def build_model(self, name, **kw):
        return M.get_model(name, **kw)

    def wrap(self, model: torch.nn.Module) -> torch.nn.Module:
        model = model.to(self.device)
        if self.world > 1:
            return DataParallel(model, bucket_mb=self.bucket_mb)
        return model

    @staticmethod
    def unwrap(model):
        return model.module if isinstance(model, DataParallel) else model

    def optimizer(self, name, params, kw):
        return make_optimizer(name, params, kw)

    # ---------------- one optimisation step ----------------
    def backward_step(self, loss, model, optimizer, zero_grad=True):
        """backward -> all-reduce completion -> (guarded) fused optimizer step. Returns False when
        the step was skipped because the loss / gradients were not finite."""
        self.step_count += 1
        s = self.step_count
        self.faults.process(s)
        loss = self.faults.loss(loss, s)
        if zero_grad:
            optimizer.zero_grad()
        guard = self.comm_watchdog.guard("backward+allreduce") if self.comm_watchdog else contextlib.nullcontext()
        with guard:
            with self.timer.phase("bwd"):
                loss.backward()
            flat = optimizer.flat_grads() if hasattr(optimizer, "flat_grads") else None
            self.faults.grads(flat[0] if flat else None, s)
            with self.timer.phase("comm"):
                if isinstance(model, DataParallel):
                    model.finish()
            ok = True
            if self.guard.should_check(s):  # same cadence on every rank: the verdict is all-reduced
                ok = self.guard.ok(loss, flat[0] if flat else None, distributed=self.world > 1)
        if ok:
            with self.timer.phase("opt"):
                gs = model.grad_scale if isinstance(model, DataParallel) else 1.0
                optimizer.step(grad_scale=gs)
        else:
            optimizer.zero_grad()
            self.log(f"[dv] non-finite loss/gradients at step {s}: step skipped ({self.guard.skipped} so far)")
        if self.watchdog is not None:
            self.watchdog.beat()
        self._track_gpu("step")
        return ok

    def _track_gpu(self, name):
        """GPU-side completion of the step just enqueued, watched by the comm watchdog: an RCCL
        all-reduce that never completes (dead / wedged peer) ends this rank even though the host
        only enqueued it (eager ``work.wait()`` is a stream wait; graph replays are one launch)."""
        # not while a graph is being captured: an event recorded in a capture cannot be queried,
        # and the watchdog thread would poll the warm-up events mid-capture (CapturedStep tracks
        # the replays instead, train_step below)
        if (self.comm_watchdog is not None and self.device.type == "cuda"
                and not torch.cuda.is_current_stream_capturing()):
            ev = torch.cuda.Event()
            ev.record()
            self.comm_watchdog.track(f"{name} {self.step_count}", ev)

    def _check_device_guard(self, optimizer):
        """Graph mode: read the device non-finite counters at the guard cadence (one sync)."""
        if not hasattr(optimizer, "device_guard_counts") or not self.guard.should_check(self.step_count):
            return
        skipped, consecutive, _ = optimizer.device_guard_counts()
        if skipped > self.guard.skipped:
            self.log(f"[dv] non-finite gradients: {skipped - self.guard.skipped} captured step(s) skipped on the device "
                     f"by step {self.step_count} ({skipped} so far)")
            self.guard.skipped = skipped
        if consecutive >= self.guard.max_consecutive:
            raise FloatingPointError(f"{consecutive} consecutive non-finite steps")

    def train_step(self, model, optimizer, forward_loss, *inputs):
        """One optimisation step: ``forward_loss(*inputs) -> (loss, extra)``, backward, all-reduce,
        optimizer step. Returns (loss, extra). With ``graph`` the step is captured on the first
        batch of each input signature and replayed (train.graph.GraphedTrainStep)."""
        def eager(*args):
            with self.timer.phase("fwd"):
                loss, extra = forward_loss(*args)
            self.backward_step(loss, model, optimizer)
            return loss, extra

        if not self.graph:
            return eager(*inputs)
        from .graph import GraphedTrainStep

        key = (id(model), id(optimizer), getattr(forward_loss, "__code__", forward_loss))
        g = self._graphed.get(key)
        if g is None:
            if hasattr(optimizer, "use_device_guard") and self.guard.every > 0:
                optimizer.use_device_guard(True)  # captured with the step: skip decided on the device
            g = self._graphed[key] = GraphedTrainStep(model, optimizer, forward_loss, eager)
        before = self.step_count
        out = g(*inputs)
        if self.step_count == before:  # replay / capture: backward_step (which counts) did not run
            self.step_count += 1
            self._track_gpu("graph replay")
        self._check_device_guard(optimizer)
        return out

    def reduce_sum(self, values):
        return D.all_reduce_scalars(list(values), device=self.device if self.device.type == "cuda" else "cpu")

    def barrier(self):
        D.barrier()

    def close(self):
        if self.watchdog is not None:
            self.watchdog.stop()
        if self.comm_watchdog is not None:
            self.comm_watchdog.stop()
        D.destroy()
