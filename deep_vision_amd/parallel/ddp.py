"""Data parallelism: bucketed gradient all-reduce overlapped with backward.

Design (MI355X-first, not a translation of DataParallel / MirroredStrategy):
  * one process per GPU; parameters live in one flat fp32 buffer laid out in reverse
    registration order (parallel.flat), gradients in a matching flat buffer;
  * buckets are contiguous slices of that gradient buffer (default 64 MB — a ring all-reduce
    over xGMI is per-link bound at ~153 GB/s, so a few large messages beat many small ones);
  * a post-accumulate-grad hook counts arrivals per bucket; the moment a bucket is complete its
    all-reduce is issued (``async_op=True``): RCCL runs it on its own stream ordered after the
    compute stream's current position, so it overlaps the rest of backward;
  * ``finish()`` (called before the optimizer) issues buckets that never completed (unused
    parameters: Inception aux heads in eval, Hourglass dead convs) and makes the compute stream
    wait on every outstanding all-reduce;
  * the 1/world averaging is fused into the optimizer kernel (``grad_scale``) — no extra pass;
  * BatchNorm statistics stay per replica (reference semantics, no SyncBN); initial parameters
    and buffers are broadcast from rank 0.
"""
from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist

from .dist import is_dist, world_size
from .flat import flatten_parameters


class _Bucket:
    __slots__ = ("start", "end", "params", "pending", "work", "issued")

    def __init__(self, start):
        self.start = start
        self.end = start
        self.params = []
        self.pending = 0
        self.work = None
        self.issued = False


class DataParallel(torch.nn.Module):
    def __init__(self, module: torch.nn.Module, bucket_mb: float = 64.0, broadcast: bool = True,
                 process_group=None, comm=None):
        super().__init__()
        self.module = module
        self.pg = process_group
        self.comm = comm  # optional injected communicator (tests): callable(tensor) -> None (sum in place)
        self.world = world_size() if comm is None else getattr(comm, "world", 1)
        self.pflat, self.gflat, layout = flatten_parameters(module, reverse=True)
        self._sync_enabled = True
        if broadcast and is_dist():
            with torch.no_grad():
                dist.broadcast(self.pflat, 0, group=self.pg)
                for b in module.buffers():
                    if b.numel():
                        dist.broadcast(b, 0, group=self.pg)
        # build buckets over the flat layout (params never split across buckets)
        cap = int(bucket_mb * 1024 * 1024 / 4)
        self.buckets = []
        cur = _Bucket(0)
        for p, off, n in layout:
            if cur.params and (cur.end - cur.start) + n > cap:
                self.buckets.append(cur)
                cur = _Bucket(off)
            cur.params.append(p)
            cur.end = off + n
        self.buckets.append(cur)
        self._bucket_of = {}
        for bi, b in enumerate(self.buckets):
            for p in b.params:
                self._bucket_of[id(p)] = bi
        self._hooks = []
        for p, _, _ in layout:
            h = self._make_hook(p)
            self._hooks.append(p.register_post_accumulate_grad_hook(h))
            # native backward kernels write gradients straight into the flat buffer and signal
            # readiness through this attribute instead of autograd's AccumulateGrad
            p._dv_ready_hook = h
        self.comm_stats = {"allreduce_calls": 0, "allreduce_bytes": 0}
        self._reset()

    # ------------------------------------------------------------------
    def _reset(self):
        for b in self.buckets:
            b.pending = len(b.params)
            b.work = None
            b.issued = False

    def _make_hook(self, p):
        pid = id(p)

        def hook(param):
            if not self._sync_enabled or self.world <= 1:
                return
            b = self.buckets[self._bucket_of[pid]]
            b.pending -= 1
            if b.pending == 0 and not b.issued:
                self._issue(b)

        return hook

    def _issue(self, b: _Bucket):
        t = self.gflat[b.start:b.end]
        b.issued = True
        self.comm_stats["allreduce_calls"] += 1
        self.comm_stats["allreduce_bytes"] += t.numel() * 4
        if self.comm is not None:
            self.comm(t)
            return
        b.work = dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)

    def forward(self, *args, **kw):
        self._reset()
        return self.module(*args, **kw)

    def prepare(self):
        """Arm the buckets for a backward pass when submodules are called directly instead of
        through ``forward`` (multi-network steps, e.g. CycleGAN's generator pair)."""
        self._reset()

    @contextlib.contextmanager
    def no_sync(self):
        """Gradient accumulation without communication (grads accumulate in the flat buffer)."""
        prev = self._sync_enabled
        self._sync_enabled = False
        try:
            yield
        finally:
            self._sync_enabled = prev

    def finish(self):
        """Issue incomplete buckets and make the current stream wait for all reductions."""
        if self.world <= 1 or not self._sync_enabled:
            return
        for b in self.buckets:
            if not b.issued:
                self._issue(b)
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()
                b.work = None

    @property
    def grad_scale(self) -> float:
        """Factor the optimizer applies to summed gradients (mean over replicas)."""
        return 1.0 / self.world

    def state_dict(self, *a, **kw):  # checkpoints never carry a `module.` prefix
        return self.module.state_dict(*a, **kw)

    def load_state_dict(self, sd, strict=True):
        return self.module.load_state_dict(sd, strict=strict)
