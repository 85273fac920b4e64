"""Tracing / profiling (the reference has none beyond wall-clock prints).

* ``StepTimer``: HIP events around named phases (fwd / bwd / comm / opt / data) of every step,
  resolved lazily (no per-step host sync), reporting ms per phase and images/s per rank; the
  node aggregate comes from one packed all-reduce.
* ``range(name)``: roctx ranges (torch.cuda.nvtx maps to roctx on ROCm) visible in rocprofv3
  ``--marker-trace`` / sys traces; a no-op on CPU.
* ``rocprof_command``: the rocprofv3 invocation used by ``--profile`` / tools/gpu_prof.sh
  (kernel trace + stats; counter collection in a separate run, never mixed with traces).
"""
from __future__ import annotations

import contextlib
import time
from collections import defaultdict
from typing import Dict, List

import torch


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors nvtx.range
    pushed = False
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        try:
            torch.cuda.nvtx.range_push(name)
            pushed = True
        except Exception:  # roctx unavailable
            pushed = False
    try:
        yield
    finally:
        if pushed:
            torch.cuda.nvtx.range_pop()


class StepTimer:
    """Per-phase device timing. ``with timer.phase('fwd'): ...`` inside ``timer.step()``."""

    def __init__(self, enabled: bool = True, device=None):
        self.cuda = enabled and torch.cuda.is_available()
        self.enabled = enabled
        self._pending: List[Dict[str, tuple]] = []
        self.totals: Dict[str, float] = defaultdict(float)
        self.counts: Dict[str, int] = defaultdict(int)
        self._cur = None
        self.samples = 0
        self.t0 = None

    @contextlib.contextmanager
    def step(self, samples: int = 0):
        self._cur = {}
        if self.t0 is None:
            self.t0 = time.perf_counter()
        try:
            yield self
        finally:
            self.samples += samples
            if self._cur:
                self._pending.append(self._cur)
            self._cur = None
            if len(self._pending) > 64:
                self.resolve()

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled or self._cur is None:
            yield
            return
        if self.cuda:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            with range(name):
                yield
            b.record()
            self._cur[name] = (a, b)
        else:
            t = time.perf_counter()
            yield
            self._cur[name] = (t, time.perf_counter())

    def resolve(self):
        if self.cuda and self._pending:
            torch.cuda.synchronize()
        for st in self._pending:
            for name, (a, b) in st.items():
                ms = a.elapsed_time(b) if self.cuda else (b - a) * 1e3
                self.totals[name] += ms
                self.counts[name] += 1
        self._pending.clear()

    def summary(self) -> Dict[str, float]:
        self.resolve()
        out = {f"{k}_ms": self.totals[k] / max(1, self.counts[k]) for k in self.totals}
        if self.t0 is not None:
            wall = time.perf_counter() - self.t0
            out["samples_per_s"] = self.samples / wall if wall > 0 else 0.0
        return out

    def reset(self):
        self.resolve()
        self.totals.clear()
        self.counts.clear()
        self.samples = 0
        self.t0 = None


def node_throughput(samples_per_s: float) -> float:
    """Sum of per-rank throughput over the process group."""
    from ..parallel.dist import all_reduce_scalars

    return all_reduce_scalars([samples_per_s])[0]


def rocprof_command(out_dir: str, argv: List[str], counters: List[str] | None = None) -> List[str]:
    """rocprofv3 invocation: kernel trace + stats, or (separately) PMC counters with stats."""
    cmd = ["rocprofv3", "--kernel-trace", "--stats", "-d", out_dir, "-o", "run"]
    if counters:
        cmd = ["rocprofv3", "--pmc", *counters, "--kernel-trace", "--stats", "-d", out_dir, "-o", "pmc"]
    return cmd + ["--", *argv]
