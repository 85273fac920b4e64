"""Data parallelism: bucketed gradient all-reduce overlapped with backward.

Replaces the reference's ``nn.DataParallel`` (R/ResNet/pytorch/train.py:353-355) and
``MirroredStrategy`` gradient all-reduce (R/YOLO/tensorflow/train.py:99-100, 281).

Design (MI355X-first, not a translation of DataParallel / MirroredStrategy):
  * one process per GPU; parameters live in one flat fp32 buffer laid out in reverse
    registration order (parallel.flat), gradients in a matching flat buffer;
  * buckets are contiguous slices of that gradient buffer (default 32 MB — a ring all-reduce
    over xGMI is per-link bound at ~153 GB/s, so a few large messages beat many small ones),
    except the last (first-layer) one, capped at ``tail_mb`` (4 MB): nothing is left to overlap
    its all-reduce, so it is kept small;
  * a parameter is *complete* when autograd's post-accumulate-grad hook fires for it. The
    engine runs a parameter's AccumulateGrad node once per backward, after EVERY node with an
    edge to it -- i.e. after the last use's backward -- even when all uses are native ops that
    accumulated straight into ``.grad`` (ops.common.grad_sink) and returned None. So a weight
    used several times in one step (CycleGAN's generators run 3x, GAN discriminators 2x)
    completes only after its last wgrad, and a bucket never starts reducing while a wgrad still
    adds into it. (Round 1 also counted a per-use native notification: every native parameter
    was reported twice and buckets were issued early.) A second report of one parameter in
    one backward raises ``DoubleReadyError`` instead of silently corrupting the bucket.
  * the moment a bucket is complete its all-reduce is issued (``async_op=True``): RCCL runs it
    on its own stream ordered after the compute stream's current position, so it overlaps the
    rest of backward. Optional bf16 wire format (``comm_dtype=torch.bfloat16``): the bucket is
    cast into a persistent bf16 staging slice, reduced, and cast back into the fp32 master
    gradient in ``finish`` (half the xGMI bytes; summation of ``world`` bf16 addends);
  * ``finish()`` (called before the optimizer) issues buckets that never completed (unused
    parameters: Inception aux heads in eval, Hourglass dead convs) and makes the compute stream
    wait on every outstanding all-reduce; with ``timing=True`` a HIP event pair around that wait
    measures the *exposed* communication time (``comm_stats['exposed_ms']``);
  * ``record_issue=True`` (overlap evidence, tests/test_ddp_gpu.py): every bucket issue records
    where it came from (a backward hook or ``finish``) and a HIP event at that point of the
    compute stream; ``finish`` records the end of backward, so ``issue_report()`` gives, per
    bucket, how much backward compute was still queued behind its all-reduce;
  * the 1/world averaging is fused into the optimizer kernel (``grad_scale``) — no extra pass;
  * BatchNorm statistics stay per replica (reference semantics, no SyncBN); initial parameters
    and buffers are broadcast from rank 0.
"""
from __future__ import annotations

import collections
import contextlib

import torch
import torch.distributed as dist

from .flat import flatten_parameters


class DoubleReadyError(RuntimeError):
    """A parameter reported a complete gradient twice in one backward (its bucket may already be
    in flight), e.g. a second ``backward(retain_graph=True)`` without a new forward / prepare."""


class _Bucket:
    __slots__ = ("start", "end", "params", "pending", "work", "issued", "wire")

    def __init__(self, start):
        self.start = start
        self.end = start
        self.params = []
        self.pending = 0
        self.work = None
        self.issued = False
        self.wire = None  # bf16 staging slice (comm_dtype != fp32)


class DataParallel(torch.nn.Module):
    def __init__(self, module: torch.nn.Module, bucket_mb: float = 32.0, broadcast: bool = True,
                 process_group=None, comm=None, comm_dtype: torch.dtype = torch.float32, timing: bool = False,
                 always_reduce: bool = False, tail_mb: float = 4.0, record_issue: bool = False):
        super().__init__()
        self.record_issue = record_issue
        self.issue_log = []  # this step's [(bucket index, 'hook' | 'finish', event | None)]
        self.bwd_end = None
        self.module = module
        self.pg = process_group
        self.comm = comm  # optional injected communicator (tests): callable(tensor) -> None (sum in place)
        pg_up = dist.is_available() and dist.is_initialized()
        if comm is not None:
            self.world = getattr(comm, "world", 1)
            self.reduce = self.world > 1
        else:
            self.world = dist.get_world_size(self.pg) if pg_up else 1
            # always_reduce: run the whole bucketed all-reduce path even on a world-1 process group
            # (exercises RCCL, the bf16 wire and HIP-graph capture of collectives on one GPU)
            self.reduce = pg_up and (self.world > 1 or always_reduce)
        self.comm_dtype = comm_dtype
        self.pflat, self.gflat, layout = flatten_parameters(module, reverse=True)
        self._sync_enabled = True
        if broadcast and self.reduce and comm is None:
            with torch.no_grad():
                dist.broadcast(self.pflat, 0, group=self.pg)
                for b in module.buffers():
                    if b.numel():
                        dist.broadcast(b, 0, group=self.pg)
        # build buckets over the flat layout (params never split across buckets). The LAST bucket
        # holds the first layers' gradients, complete only at the very end of backward: its
        # all-reduce cannot overlap anything, so it is capped at tail_mb (the rest of the tail
        # moves into the bucket before it, which still overlaps the stem's wgrad).
        cap = max(1, int(bucket_mb * 1024 * 1024 / 4))
        tail_cap = max(1, int(min(bucket_mb, tail_mb) * 1024 * 1024 / 4))
        total = self.gflat.numel()
        self.buckets = []
        cur = _Bucket(0)
        for p, off, n in layout:
            in_tail = off >= total - tail_cap
            if cur.params and ((cur.end - cur.start) + n > cap or (in_tail and cur.start < total - tail_cap)):
                self.buckets.append(cur)
                cur = _Bucket(off)
            cur.params.append(p)
            cur.end = off + n
        self.buckets.append(cur)
        if comm_dtype != torch.float32:
            self._wire = torch.empty(self.gflat.numel(), dtype=comm_dtype, device=self.gflat.device)
            for b in self.buckets:
                b.wire = self._wire[b.start:b.end]
        self._bucket_of = {}
        self.params = [p for p, _, _ in layout]
        for bi, b in enumerate(self.buckets):
            for p in b.params:
                self._bucket_of[id(p)] = bi
        self._hooks = []
        for p in self.params:
            self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(p)))
        self.timing = timing and self.gflat.is_cuda
        self.comm_stats = {"allreduce_calls": 0, "allreduce_bytes": 0, "steps": 0,
                           # bounded: one HIP event pair per step (an unbounded list leaks)
                           "exposed_ms": collections.deque(maxlen=1024)}
        self._reset()

    # ------------------------------------------------------------------ readiness
    def _reset(self):
        for b in self.buckets:
            b.pending = len(b.params)
            b.work = None
            b.issued = False
        self._done = set()
        self.issue_log = []
        self.bwd_end = None

    def _make_hook(self, p):
        pid = id(p)
        bi = self._bucket_of[pid]

        def hook(param):
            if not self._sync_enabled or not self.reduce:
                return
            if pid in self._done:
                raise DoubleReadyError(f"parameter {tuple(param.shape)} reported ready twice in one backward "
                                       "(retain_graph double backward without a new forward/prepare?)")
            self._done.add(pid)
            b = self.buckets[bi]
            b.pending -= 1
            if b.pending == 0 and not b.issued:
                self._issue(b, "hook")

        return hook

    # ------------------------------------------------------------------ communication
    def _issue(self, b: _Bucket, where: str = "finish"):
        side = None
        if self.gflat.is_cuda:  # weight gradients still queued on the side stream (ops.conv)
            from ..ops.conv import wgrad_side_comm_stream

            side = wgrad_side_comm_stream()
        if side is not None:
            with torch.cuda.stream(side):
                return self._issue_on(b, where)
        return self._issue_on(b, where)

    def _issue_on(self, b: _Bucket, where: str):
        t = self.gflat[b.start:b.end]
        b.issued = True
        self.comm_stats["allreduce_calls"] += 1
        if self.record_issue:
            ev = None
            if t.is_cuda and not torch.cuda.is_current_stream_capturing():
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
            self.issue_log.append((self.buckets.index(b), where, ev))
        if self.comm is not None:
            self.comm_stats["allreduce_bytes"] += t.numel() * 4
            self.comm(t)
            return
        from ..profiling import range as prange

        with prange(f"dv_allreduce[{b.start}:{b.end}]"):
            if b.wire is not None:
                b.wire.copy_(t)
                t = b.wire
            self.comm_stats["allreduce_bytes"] += t.numel() * t.element_size()
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
        if not self.reduce or not self._sync_enabled:
            return
        if self.record_issue and self.gflat.is_cuda and not torch.cuda.is_current_stream_capturing():
            self.bwd_end = torch.cuda.Event(enable_timing=True)
            self.bwd_end.record()
        for b in self.buckets:
            if not b.issued:
                self._issue(b, "finish")
        ev = None
        if self.timing and not torch.cuda.is_current_stream_capturing():
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()
                b.work = None
                if b.wire is not None:
                    self.gflat[b.start:b.end].copy_(b.wire)
        self.comm_stats["steps"] += 1
        if ev is not None:
            ev[1].record()
            self.comm_stats["exposed_ms"].append(ev)

    def issue_report(self):
        """[(bucket, 'hook' | 'finish', MB, ms of backward compute queued after the issue)] of the
        last step (record_issue=True; synchronises)."""
        torch.cuda.synchronize()
        out = []
        for bi, where, ev in self.issue_log:
            b = self.buckets[bi]
            ms = ev.elapsed_time(self.bwd_end) if (ev is not None and self.bwd_end is not None) else None
            out.append((bi, where, (b.end - b.start) * 4 / 2 ** 20, ms))
        return out

    def exposed_comm_ms(self, last: int | None = None) -> float:
        """Mean compute-stream time spent waiting on gradient all-reduces (synchronises)."""
        evs = list(self.comm_stats["exposed_ms"])
        if last:
            evs = evs[-last:]
        if not evs:
            return 0.0
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in evs) / len(evs)

    @property
    def grad_scale(self) -> float:
        """Factor the optimizer applies to summed gradients (mean over replicas)."""
        return 1.0 / self.world

    def state_dict(self, *a, **kw):  # checkpoints never carry a `module.` prefix
        return self.module.state_dict(*a, **kw)

    def load_state_dict(self, sd, strict=True):
        return self.module.load_state_dict(sd, strict=strict)
