"""Distributed data parallelism on CPU (gloo, world size 2; SURVEY §7.5 4a/4b semantics).

* DP-2 over half batches == one process over the full batch (BN-free model: identical gradient
  averaging and identical optimizer updates, incl. the fused 1/world grad scale)
* bucket bookkeeping: several buckets, every one issued once per step; unused parameters do
  not deadlock (issued in ``finish``); ``no_sync`` accumulation
* broadcast of initial parameters from rank 0
* packed scalar all-reduce
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(16, 64)
        self.b = torch.nn.Linear(64, 64)
        self.unused = torch.nn.Linear(8, 8)  # never receives a gradient
        self.c = torch.nn.Linear(64, 4)

    def forward(self, x):
        return self.c(torch.tanh(self.b(torch.relu(self.a(x)))))


def _worker(rank, world, port, q, order="ddp_first"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from deep_vision_amd.parallel.ddp import DataParallel
    from deep_vision_amd.parallel.dist import all_reduce_scalars, init_distributed
    from deep_vision_amd.train.optim import FusedSGD

    init_distributed("gloo")
    torch.manual_seed(100 + rank)  # different init per rank: broadcast must fix it
    net = Net()
    if order == "opt_first":  # the optimizer flattens first; DataParallel re-lays the params out
        opt = FusedSGD(net.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
        ddp = DataParallel(net, bucket_mb=0.01)
    else:
        ddp = DataParallel(net, bucket_mb=0.01)  # tiny buckets -> several all-reduces
        opt = FusedSGD(ddp.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    g = torch.Generator().manual_seed(0)
    xs = [torch.randn(8, 16, generator=g) for _ in range(3)]
    ys = [torch.randn(8, 4, generator=g) for _ in range(3)]
    for x, y in zip(xs, ys):
        xl, yl = x[rank * 4:(rank + 1) * 4], y[rank * 4:(rank + 1) * 4]
        opt.zero_grad()
        loss = ((ddp(xl) - yl) ** 2).mean()
        loss.backward()
        ddp.finish()
        opt.step(grad_scale=ddp.grad_scale)
    issued = ddp.comm_stats["allreduce_calls"]
    # no_sync: local accumulation only
    with ddp.no_sync():
        opt.zero_grad()
        ((ddp(xs[0][rank * 4:(rank + 1) * 4]) - ys[0][rank * 4:(rank + 1) * 4]) ** 2).mean().backward()
        ddp.finish()
    s = all_reduce_scalars([float(rank + 1)], device="cpu")[0]
    # numpy copies: pickled by value (tensors would be shared through fds of an exiting process)
    # the optimizer must update the very buffer DataParallel reduces into
    assert opt._flat[0]["param"].data_ptr() == ddp.pflat.data_ptr()
    assert opt._flat[0]["grad"].data_ptr() == ddp.gflat.data_ptr()
    q.put((rank, {k: v.detach().numpy().copy() for k, v in net.state_dict().items()}, issued, len(ddp.buckets), s,
           net.a.weight.grad.numpy().copy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("order", ["ddp_first", "opt_first"])
def test_ddp_gloo_matches_single_process(order):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, order)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=240)
        res[r[0]] = r[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sd0, issued, nb, s, _ = res[0]
    sd1 = res[1][0]
    sd0 = {k: torch.from_numpy(v) for k, v in sd0.items()}
    sd1 = {k: torch.from_numpy(v) for k, v in sd1.items()}
    for k in sd0:
        assert torch.equal(sd0[k], sd1[k]), k  # replicas stay identical
    assert nb >= 3 and issued == 3 * nb  # every bucket issued exactly once per step
    assert s == 3.0
    # reference: one process, full batch, same (rank-0) initial weights
    from deep_vision_amd.train.optim import FusedSGD

    torch.manual_seed(100)
    ref = Net()
    opt = FusedSGD(ref.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    g = torch.Generator().manual_seed(0)
    xs = [torch.randn(8, 16, generator=g) for _ in range(3)]
    ys = [torch.randn(8, 4, generator=g) for _ in range(3)]
    for x, y in zip(xs, ys):
        opt.zero_grad()
        ((ref(x) - y) ** 2).mean().backward()
        opt.step()
    for k, v in ref.state_dict().items():
        assert torch.allclose(sd0[k], v, atol=1e-6, rtol=1e-5), k
    # no_sync left the two ranks' gradients different (local halves)
    assert not torch.allclose(torch.from_numpy(res[0][4]), torch.from_numpy(res[1][4]))


def _trainer_worker(rank, world, port, tmp, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from deep_vision_amd.config import get_config
    from deep_vision_amd.train.classification import run_epochs

    last, loggers = run_epochs(get_config("lenet5"), None, device="cpu", synthetic=True, synthetic_size=128,
                               num_workers=0, checkpoint_dir=tmp + "/", epochs=1, max_steps=3, val_steps=1)
    q.put((rank, last, loggers["val_loss"]["value"]))


def test_classification_trainer_two_ranks(tmp_path):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_trainer_worker, args=(r, world, port, str(tmp_path), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=300) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][0] is not None and res[1][0] is None  # rank 0 writes the checkpoint
    assert res[0][1] == pytest.approx(res[1][1])  # validation metrics are all-reduced


# ---------------------------------------------------------------------------------------------
# Use accounting for native gradient sinks: a weight used several times in one
# step must complete only after its LAST use. On CPU the native sink path is emulated by an
# autograd.Function that accumulates into .grad exactly like ops/conv.py's wgrad kernels.
# ---------------------------------------------------------------------------------------------
_FORCE_FALLBACK = [False]


class _SinkLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return x @ w.t()

    @staticmethod
    def backward(ctx, dy):
        from deep_vision_amd.ops.common import grad_sink

        x, w = ctx.saved_tensors
        dw = dy.t() @ x
        sink = None if _FORCE_FALLBACK[0] else grad_sink(w)
        if sink is not None:
            sink.add_(dw)
            dw = None
        return dy @ w, dw


def _sink_linear(x, w):
    return _SinkLinearFn.apply(x, w)


class _SharedNet(torch.nn.Module):
    """One weight applied three times (CycleGAN-style reuse) plus a plain torch layer."""

    def __init__(self):
        super().__init__()
        self.shared = torch.nn.Parameter(torch.randn(16, 16) * 0.2)
        self.head = torch.nn.Linear(16, 4)

    def forward(self, x):
        for _ in range(3):
            x = torch.tanh(_sink_linear(x, self.shared))
        return self.head(x)


class _RecordingComm:
    world = 2

    def __init__(self):
        self.snaps = []

    def __call__(self, t):
        self.snaps.append((t.data_ptr(), t.clone()))


def test_ddp_multi_use_completes_after_last_use():
    from deep_vision_amd.parallel.ddp import DataParallel

    torch.manual_seed(0)
    net = _SharedNet()
    comm = _RecordingComm()
    ddp = DataParallel(net, bucket_mb=16 * 16 * 4 / 2**20, comm=comm)  # the shared weight gets its own bucket
    x = torch.randn(8, 16)
    for _ in range(2):
        for p in net.parameters():
            p.grad.zero_()
        comm.snaps.clear()
        ddp(x).sum().backward()
        ddp.finish()
        # every bucket issued exactly once, and what was on the wire is the FINAL gradient
        assert len(comm.snaps) == len(ddp.buckets)
        for b in ddp.buckets:
            t = ddp.gflat[b.start:b.end]
            snap = [s for ptr, s in comm.snaps if ptr == t.data_ptr()]
            assert len(snap) == 1 and torch.equal(snap[0], t)
    # reference gradient (plain autograd, no sinks)
    ref = _SharedNet()
    ref.load_state_dict(net.state_dict())
    y = x
    for _ in range(3):
        y = torch.tanh(y @ ref.shared.t())
    ref.head(y).sum().backward()
    assert torch.allclose(net.shared.grad, ref.shared.grad, atol=1e-5)


def test_ddp_double_report_raises():
    """A second backward through the same graph without a new forward reports every parameter
    again: the guard refuses instead of re-issuing buckets into live gradients."""
    from deep_vision_amd.parallel.ddp import DataParallel, DoubleReadyError

    net = _SharedNet()
    ddp = DataParallel(net, comm=_RecordingComm())
    loss = ddp(torch.randn(4, 16)).sum()
    loss.backward(retain_graph=True)
    with pytest.raises(DoubleReadyError):
        loss.backward()


def test_ddp_fallback_use_waits_for_autograd():
    """A native use whose gradient goes back through autograd (no sink) completes only when
    AccumulateGrad has run."""
    from deep_vision_amd.parallel.ddp import DataParallel

    net = _SharedNet()
    comm = _RecordingComm()
    ddp = DataParallel(net, bucket_mb=16 * 16 * 4 / 2**20, comm=comm)
    x = torch.randn(4, 16)
    _FORCE_FALLBACK[0] = True  # every native use hands its gradient back to autograd
    try:
        ddp(x).sum().backward()
    finally:
        _FORCE_FALLBACK[0] = False
    ddp.finish()
    b = ddp.buckets[ddp._bucket_of[id(net.shared)]]
    t = ddp.gflat[b.start:b.end]
    assert t.abs().sum() > 0
    snap = [s for ptr, s in comm.snaps if ptr == t.data_ptr()]
    assert len(snap) == 1 and torch.equal(snap[0], t)


def _fault_worker(rank, world, port, spec):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), DV_FAULT=spec, DV_COMM_TIMEOUT="20")
    from deep_vision_amd.parallel.ddp import DataParallel
    from deep_vision_amd.parallel.dist import init_distributed
    from deep_vision_amd.parallel.watchdog import CommWatchdog
    from deep_vision_amd.utils.fault import FaultInjector

    init_distributed("gloo", timeout_s=30)
    wd = CommWatchdog(timeout=20).start()
    net = Net()
    ddp = DataParallel(net, bucket_mb=0.01)
    inj = FaultInjector(rank=rank)
    for step in range(1, 6):
        inj.process(step)
        with wd.guard("allreduce"):
            ddp(torch.randn(4, 16)).sum().backward()
            ddp.finish()
    os._exit(0)


def test_kill_rank_tears_down_every_rank():
    """DV_FAULT=kill_rank@3:1 -> rank 1 dies at step 3; rank 0 must not hang: its collective
    fails (or the comm watchdog fires) and it exits non-zero within the timeout."""
    import time

    world = 2
    ctx = mp.get_context("spawn")
    port = _port()
    procs = [ctx.Process(target=_fault_worker, args=(r, world, port, "kill_rank@3:1")) for r in range(world)]
    t0 = time.time()
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert all(c is not None and c != 0 for c in codes), codes
    assert time.time() - t0 < 120


def _nan_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from deep_vision_amd.parallel.ddp import DataParallel
    from deep_vision_amd.parallel.dist import init_distributed
    from deep_vision_amd.train.optim import FusedSGD
    from deep_vision_amd.utils.fault import FaultInjector, NonFiniteGuard

    init_distributed("gloo")
    torch.manual_seed(0)
    net = Net()
    ddp = DataParallel(net, bucket_mb=0.01)
    opt = FusedSGD(ddp.parameters(), lr=0.1)
    guard = NonFiniteGuard(every=1)
    inj = FaultInjector("inf_grad@2:1", rank=rank)  # only rank 1 sees a bad gradient
    decisions = []
    for step in range(1, 5):
        opt.zero_grad()
        ddp(torch.randn(4, 16)).sum().backward()
        inj.grads(ddp.gflat, step)
        ddp.finish()
        ok = guard.ok(torch.zeros(()), ddp.gflat, distributed=True)
        decisions.append(ok)
        if ok:
            opt.step(grad_scale=ddp.grad_scale)
    q.put((rank, decisions, net.a.weight.detach().numpy().copy()))
    dist.destroy_process_group()


def test_nan_skip_decision_identical_across_ranks():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_nan_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=240) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][0] == res[1][0] == [True, False, True, True]
    assert (res[0][1] == res[1][1]).all()  # replicas still identical after the skipped step


class _NeverDone:
    """Stands in for a torch.cuda.Event recorded after a replay whose all-reduce never completes."""

    def query(self):
        return False


class _DoneAfter:
    def __init__(self, n):
        self.n = n

    def query(self):
        self.n -= 1
        return self.n < 0


def test_comm_watchdog_event_deadline_hook():
    """GPU work tracked by event (graph replays) that never completes fires
    the watchdog with EXIT_COMM_TIMEOUT; completed events are dropped in order."""
    import time

    from deep_vision_amd.parallel.watchdog import EXIT_COMM_TIMEOUT, CommWatchdog

    fired = []
    wd = CommWatchdog(timeout=0.3, poll=0.05, on_timeout=lambda c, why: fired.append((c, why)))
    wd.track("done soon", _DoneAfter(2))
    wd.start()
    time.sleep(0.5)
    assert not fired and wd.pending() == 0
    wd.track("graph replay 7", _NeverDone())
    t0 = time.time()
    while not fired and time.time() - t0 < 5:
        time.sleep(0.05)
    wd.stop()
    assert fired and fired[0][0] == EXIT_COMM_TIMEOUT and "graph replay 7" in fired[0][1]


def test_comm_watchdog_event_deadline_exits_process():
    """Without a hook the rank ends itself with os._exit(EXIT_COMM_TIMEOUT) -- no Python cleanup
    that could block on a wedged communicator."""
    import subprocess
    import sys
    import time

    from deep_vision_amd.parallel.watchdog import EXIT_COMM_TIMEOUT

    code = ("import time, sys; sys.path.insert(0, %r)\n"
            "from deep_vision_amd.parallel.watchdog import CommWatchdog\n"
            "class E:\n    def query(self): return False\n"
            "wd = CommWatchdog(timeout=0.5, poll=0.05).start()\n"
            "wd.track('graph replay 3', E())\n"
            "time.sleep(30)\n") % os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    t0 = time.time()
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == EXIT_COMM_TIMEOUT, (r.returncode, r.stderr[-500:])
    assert time.time() - t0 < 20
    assert "graph replay 3" in r.stderr


def test_comm_watchdog_event_error_is_comm_error():
    from deep_vision_amd.parallel.watchdog import EXIT_COMM_ERROR, CommWatchdog

    class Boom:
        def query(self):
            raise RuntimeError("HIP error: the launch failed")

    fired = []
    wd = CommWatchdog(timeout=60, poll=0.05, on_timeout=lambda c, why: fired.append((c, why)))
    wd.track("step 1", Boom())
    late = wd._check_events(0.0)
    assert late is not None and "launch failed" in late[2]
    wd.start()
    import time

    t0 = time.time()
    while not fired and time.time() - t0 < 5:
        time.sleep(0.05)
    wd.stop()
    assert fired and fired[0][0] == EXIT_COMM_ERROR
