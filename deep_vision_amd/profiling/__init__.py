"""Tracing / profiling (the reference has none beyond wall-clock prints).

* ``StepTimer``: HIP events around named phases (fwd / bwd / comm / opt / data) of every step,
  resolved lazily (no per-step host sync), reporting ms per phase and images/s per rank; the
  node aggregate comes from one packed all-reduce.
* ``range(name)``: roctx ranges (torch.cuda.nvtx maps to roctx on ROCm) visible in rocprofv3
  ``--marker-trace`` / sys traces; a no-op on CPU.
* ``rocprof_command``: the rocprofv3 invocations used by ``--profile rocprof`` / tools/gpu.sh:
  kernel trace + stats, or (a separate run per counter group) ``--pmc`` counters with nothing
  but the counter collection -- never combined with traces.
* ``run_under_rocprof``: ``--profile rocprof`` on any entry point re-runs the same command as a
  child of ``rocprofv3 --kernel-trace --stats`` (the program itself directly after ``--``, no
  shell or env hop) before anything touches the GPU, and exits with the child's status.
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
    """rocprofv3 invocation: kernel trace + stats (per-kernel times), or -- in its own run --
    PMC counters alone (``--pmc`` is never combined with a trace domain)."""
    if counters:
        return ["rocprofv3", "--pmc", *counters, "-d", out_dir, "-o", "pmc", "--output-format", "csv", "--", *argv]
    return ["rocprofv3", "--kernel-trace", "--stats", "-d", out_dir, "-o", "run", "--output-format", "csv", "--",
            *argv]


def run_under_rocprof(argv: List[str] | None = None, out_dir: str | None = None) -> None:
    """Re-run this program (``sys.argv`` without the ``--profile rocprof`` flag) under rocprofv3
    kernel tracing as a child process and exit with its status. Must be called before any GPU
    work in this process (nothing is exec'ed from a GPU-initialised process)."""
    import os
    import subprocess
    import sys

    args = list(sys.argv if argv is None else [sys.argv[0]] + list(argv))
    clean, skip = [], False
    for a in args:
        if skip:
            skip = False
            if a in ("timer", "rocprof"):
                continue
        if a == "--profile":
            skip = True
            continue
        if a.startswith("--profile="):
            continue
        clean.append(a)
    out_dir = out_dir or os.environ.get("DV_ROCPROF_DIR", os.path.abspath("rocprof_out"))
    script = os.path.abspath(clean[0])
    cmd = rocprof_command(out_dir, [sys.executable, script] + clean[1:])
    print("[dv-profile] " + " ".join(cmd), flush=True)
    sys.exit(subprocess.call(cmd))
