"""Failure detection and fault injection (the reference only skips NaN validation
batches in Hourglass, R/Hourglass/tensorflow/train.py:126-130).

* ``NonFiniteGuard``: loss / gradient non-finite detection with skip-step. Checking costs a
  device->host sync, so it runs every ``every`` steps (default: the logging cadence) unless
  ``DV_NAN_CHECK=step``; a skipped step zeroes the gradients and leaves parameters and optimizer
  state untouched; ``max_consecutive`` skips abort the run.
* ``Watchdog``: a heartbeat thread; if no step completes within ``timeout`` seconds (a hung
  collective, a wedged kernel) it dumps every thread's stack and aborts the process so the
  launcher tears the job down instead of hanging (torch.distributed's own timeout covers the
  RCCL side).
* ``FaultInjector``: ``DV_FAULT="nan_loss@5,kill_rank@10:1,hang@20:0"`` -- deterministic faults
  for tests of the above.
"""
from __future__ import annotations

import faulthandler
import math
import os
import sys
import threading
import time

import torch


class NonFiniteGuard:
    def __init__(self, every: int = 10, max_consecutive: int = 10):
        mode = os.environ.get("DV_NAN_CHECK", "")
        self.every = 1 if mode == "step" else (0 if mode == "off" else every)
        self.max_consecutive = max_consecutive
        self.skipped = 0
        self.consecutive = 0

    def should_check(self, step: int) -> bool:
        return self.every > 0 and step % self.every == 0

    def ok(self, loss: torch.Tensor, grads: torch.Tensor | None = None, distributed: bool = False) -> bool:
        """True if finite. ``grads`` may be the flat gradient buffer (one fused reduction).
        ``distributed``: the verdict is all-reduced (MAX of the non-finite flag) so every rank
        skips or steps together -- a NaN loss seen by one rank only must not fork the replicas."""
        vals = [loss.detach().float().reshape(1).to(grads.device if grads is not None else loss.device)]
        if grads is not None:
            vals.append(grads.detach().float().abs().sum().reshape(1))
        bad = (~torch.isfinite(torch.cat(vals))).any().to(torch.float32).reshape(1)
        if distributed:
            from ..parallel.dist import is_dist

            if is_dist():
                import torch.distributed as dist

                dist.all_reduce(bad, op=dist.ReduceOp.MAX)
        finite = not bool(bad.item())
        if finite:
            self.consecutive = 0
            return True
        self.skipped += 1
        self.consecutive += 1
        if self.consecutive >= self.max_consecutive:
            raise FloatingPointError(f"{self.consecutive} consecutive non-finite steps")
        return False


class Watchdog:
    def __init__(self, timeout: float = 1800.0, on_timeout=None):
        self.timeout = timeout
        self.on_timeout = on_timeout
        self._last = time.monotonic()
        self._stop = threading.Event()
        self._t = None

    def start(self):
        if self.timeout and self.timeout > 0 and self._t is None:
            self._t = threading.Thread(target=self._run, name="dv-watchdog", daemon=True)
            self._t.start()
        return self

    def beat(self):
        self._last = time.monotonic()

    def stop(self):
        self._stop.set()

    def _run(self):
        while not self._stop.wait(min(5.0, self.timeout / 4)):
            if time.monotonic() - self._last > self.timeout:
                sys.stderr.write(f"[dv-watchdog] no training progress for {self.timeout:.0f}s; dumping stacks\n")
                faulthandler.dump_traceback(all_threads=True)
                if self.on_timeout is not None:
                    self.on_timeout()
                else:
                    os._exit(3)
                return


class FaultInjector:
    """Parses ``DV_FAULT``: comma-separated ``kind@step[:rank]``; kinds nan_loss, inf_grad,
    kill_rank, hang."""

    def __init__(self, spec: str | None = None, rank: int = 0):
        spec = os.environ.get("DV_FAULT", "") if spec is None else spec
        self.rank = rank
        self.faults = []
        for item in filter(None, (s.strip() for s in spec.split(","))):
            kind, _, rest = item.partition("@")
            step, _, r = rest.partition(":")
            self.faults.append((kind, int(step), int(r) if r else None))

    def _hit(self, kind, step):
        return any(k == kind and s == step and (r is None or r == self.rank) for k, s, r in self.faults)

    def loss(self, loss: torch.Tensor, step: int) -> torch.Tensor:
        if self._hit("nan_loss", step):
            return loss * float("nan")
        return loss

    def grads(self, flat_grad: torch.Tensor | None, step: int):
        if flat_grad is not None and self._hit("inf_grad", step):
            flat_grad.view(-1)[0] = math.inf

    def process(self, step: int):
        if self._hit("kill_rank", step):
            sys.stderr.write(f"[dv-fault] killing rank {self.rank} at step {step}\n")
            sys.stderr.flush()
            os._exit(17)
        if self._hit("hang", step):
            time.sleep(1e9)
