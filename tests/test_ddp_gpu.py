"""Data parallelism through the NATIVE kernels on the GPU.

* two gloo ranks sharing one MI355X: a conv weight used twice per step (native wgrad sinks into
  the flat gradient buffer twice) -> the all-reduced gradient equals the single-process
  full-batch gradient (the bucket must not start before the second use);
* RCCL (``nccl`` backend) DP-2 on two GPUs (skipped on a 1-GPU box): same check + initial
  parameter broadcast + every bucket issued exactly once + a never-used parameter.
"""
import os
import queue
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _make_net():
    from deep_vision_amd import nn

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.stem = nn.Conv2d(16, 64, 3, padding=1, bias=False)
            self.shared = nn.Conv2d(64, 64, 3, padding=1, bias=False)  # applied twice
            self.unused = nn.Conv2d(64, 64, 1, bias=False)  # never used: finish() must issue it
            self.fc = nn.Linear(64, 10)

        def forward(self, x):
            from deep_vision_amd import ops as F

            x = F.relu(self.stem(x))
            x = F.relu(self.shared(x))
            x = F.relu(self.shared(x))
            return self.fc(x.float().mean((2, 3)))

    return Net()


def _data(world, rank, dev):
    g = torch.Generator().manual_seed(11)
    x = torch.randn(8 * world, 16, 16, 16, generator=g)
    y = torch.randint(0, 10, (8 * world,), generator=g)
    if rank is None:
        return x.to(dev), y.to(dev)
    return x[rank * 8:(rank + 1) * 8].to(dev), y[rank * 8:(rank + 1) * 8].to(dev)


def _worker(rank, world, port, backend, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), DV_DIST_BACKEND=backend)
    import torch.distributed as dist

    from deep_vision_amd import ops as F
    from deep_vision_amd.parallel.ddp import DataParallel
    from deep_vision_amd.parallel.dist import init_distributed
    from deep_vision_amd.train.optim import FusedSGD

    _, _, _, dev = init_distributed(backend)
    torch.manual_seed(5 + rank)  # different init per rank: the broadcast must fix it
    net = _make_net().to(dev)
    ddp = DataParallel(net, bucket_mb=0.05)
    opt = FusedSGD(net.parameters(), lr=0.01)
    x, y = _data(world, rank, dev)
    opt.zero_grad()
    F.cross_entropy(ddp(x), y).backward()
    ddp.finish()
    g = (ddp.gflat * ddp.grad_scale).cpu().numpy().copy()
    p0 = ddp.pflat.cpu().numpy().copy()
    q.put((rank, g, p0, ddp.comm_stats["allreduce_calls"], len(ddp.buckets)))
    dist.destroy_process_group()


def _run(backend, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, backend, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=180) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _reference(p0):
    """Single process, full batch, the broadcast (rank-0) parameters."""
    from deep_vision_amd import ops as F
    from deep_vision_amd.parallel.flat import flatten_parameters

    dev = torch.device("cuda:0")
    net = _make_net().to(dev)
    pflat, gflat, _ = flatten_parameters(net, reverse=True)
    with torch.no_grad():
        pflat.copy_(torch.from_numpy(p0))
    x, y = _data(2, None, dev)
    F.cross_entropy(net(x), y).backward()
    return gflat.cpu()


def _check(res, world):
    g0, p0, calls, nb = res[0]
    for r in range(1, world):
        assert (res[r][1] == p0).all(), "initial parameters were not broadcast"
        assert (res[r][0] == g0).all(), "replicas hold different reduced gradients"
    assert nb >= 3 and calls == nb, (calls, nb)  # every bucket issued exactly once (incl. the unused one)
    ref = _reference(p0)
    g = torch.from_numpy(g0)
    err = (g - ref).norm() / ref.norm()
    assert err < 3e-2, float(err)


def test_gloo_ranks_share_gpu_multi_use_weight():
    _check(_run("gloo", 2), 2)


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="RCCL DP needs >= 2 GPUs")
def test_rccl_dp2_matches_single_process():
    _check(_run("nccl", 2), 2)


# ------------------------------------------------------------------------------------------------
# Multi-step trajectories: the optimizer must update the buffer DataParallel
# reduces into whichever order the two were built in, through the native kernels.
# ------------------------------------------------------------------------------------------------
STEPS = 5


def _traj_worker(rank, world, port, backend, order, comm_dtype, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), DV_DIST_BACKEND=backend)
    import torch.distributed as dist

    from deep_vision_amd import ops as F
    from deep_vision_amd.parallel.ddp import DataParallel
    from deep_vision_amd.parallel.dist import init_distributed
    from deep_vision_amd.train.optim import FusedSGD

    _, _, _, dev = init_distributed(backend, force=True)
    torch.manual_seed(5)
    net = _make_net().to(dev)
    p0 = torch.cat([p.detach().reshape(-1).cpu() for p in net.parameters()])
    kw = dict(bucket_mb=0.05, always_reduce=True, comm_dtype=comm_dtype)
    if order == "opt_first":
        opt = FusedSGD(net.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
        ddp = DataParallel(net, **kw)
    else:
        ddp = DataParallel(net, **kw)
        opt = FusedSGD(net.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    x, y = _data(world, rank, dev)
    losses = []
    for _ in range(STEPS):
        opt.zero_grad()
        loss = F.cross_entropy(ddp(x), y)
        loss.backward()
        ddp.finish()
        opt.step(grad_scale=ddp.grad_scale)
        losses.append(float(loss))
    torch.cuda.synchronize()
    assert opt._flat[0]["param"].data_ptr() == ddp.pflat.data_ptr()
    p = torch.cat([p.detach().reshape(-1).cpu() for p in net.parameters()])
    q.put((rank, p0.numpy(), p.numpy(), losses, ddp.comm_stats["allreduce_calls"], len(ddp.buckets)))
    dist.destroy_process_group()


def _run_traj(backend, world, order, comm_dtype=torch.float32):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_traj_worker, args=(r, world, port, backend, order, comm_dtype, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=180) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _single_traj(world):
    """One process, no DataParallel, the global batch."""
    from deep_vision_amd import ops as F
    from deep_vision_amd.train.optim import FusedSGD

    dev = torch.device("cuda:0")
    torch.manual_seed(5)
    net = _make_net().to(dev)
    opt = FusedSGD(net.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    x, y = _data(world, None, dev)
    losses = []
    for _ in range(STEPS):
        opt.zero_grad()
        loss = F.cross_entropy(net(x), y)
        loss.backward()
        opt.step()
        losses.append(float(loss))
    torch.cuda.synchronize()
    return torch.cat([p.detach().reshape(-1).cpu() for p in net.parameters()]), losses


@pytest.mark.parametrize("order", ["ddp_first", "opt_first"])
def test_gloo_dp2_five_step_trajectory(order):
    res = _run_traj("gloo", 2, order)
    p0, p, losses, calls, nb = res[0]
    assert (res[1][1] == p).all(), "replicas diverged"
    assert calls == STEPS * nb
    ref, ref_losses = _single_traj(2)
    p0 = torch.from_numpy(p0)
    d, dref = torch.from_numpy(p) - p0, ref - p0
    assert dref.norm() > 0 and d.norm() > 0.5 * dref.norm(), "the DP model did not move"
    err = (d - dref).norm() / dref.norm()
    assert err < 5e-2, float(err)
    glob = [(a + b) / 2 for a, b in zip(losses, res[1][2])]
    assert glob[-1] < glob[0]
    assert glob[-1] == pytest.approx(ref_losses[-1], rel=2e-2)


@pytest.mark.parametrize("comm_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("order", ["ddp_first", "opt_first"])
def test_rccl_world1_bucket_path(order, comm_dtype):
    """A world-1 ``nccl`` (RCCL) process group with DataParallel forced on: every bucket goes
    through the async RCCL all-reduce (and the bf16 wire), five steps track the plain run."""
    res = _run_traj("nccl", 1, order, comm_dtype)
    p0, p, losses, calls, nb = res[0]
    assert calls == STEPS * nb and nb >= 3
    ref, ref_losses = _single_traj(1)
    p0 = torch.from_numpy(p0)
    d, dref = torch.from_numpy(p) - p0, ref - p0
    err = (d - dref).norm() / dref.norm()
    assert err < (1e-3 if comm_dtype == torch.float32 else 2e-2), float(err)
    assert losses[-1] < losses[0]


def _overlap_worker(port, q):
    """ResNet-50 on the native kernels, world-1 RCCL group, DataParallel forced on: where was each
    bucket's all-reduce issued, and how much backward compute was still queued behind it."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    import torch.distributed as dist

    from deep_vision_amd import ops as F
    from deep_vision_amd.models import ResNet50
    from deep_vision_amd.parallel.ddp import DataParallel
    from deep_vision_amd.parallel.dist import init_distributed
    from deep_vision_amd.train.optim import FusedSGD

    init_distributed("nccl", force=True)
    torch.manual_seed(0)
    m = ResNet50().cuda()
    ddp = DataParallel(m, bucket_mb=8, always_reduce=True, record_issue=True)
    opt = FusedSGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    x = torch.randn(64, 3, 160, 160, device="cuda")
    y = torch.randint(0, 1000, (64,), device="cuda")
    for _ in range(3):
        opt.zero_grad()
        loss = F.cross_entropy(ddp(x), y)
        b0 = torch.cuda.Event(enable_timing=True)
        b0.record()
        loss.backward()
        ddp.finish()
        opt.step(grad_scale=ddp.grad_scale)
    rep = ddp.issue_report()
    bwd_ms = b0.elapsed_time(ddp.bwd_end)
    q.put((rep, bwd_ms, len(ddp.buckets)))
    dist.destroy_process_group()


def test_bucket_allreduce_overlaps_backward():
    """every bucket's all-reduce is issued from a backward
    hook, in bucket order, while backward compute is still queued behind it -- not by finish()."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_overlap_worker, args=(_port(), q))
    p.start()
    rep = None
    for _ in range(110):  # a worker that dies fails the test now, not at a 300 s queue timeout
        try:
            rep, bwd_ms, nb = q.get(timeout=1)
            break
        except queue.Empty:
            if not p.is_alive():
                break
    assert rep is not None, f"worker exited with {p.exitcode} before reporting"
    p.join(timeout=60)
    assert p.exitcode == 0
    assert nb >= 8 and len(rep) == nb
    assert all(where == "hook" for _, where, _, _ in rep), rep
    assert [bi for bi, _, _, _ in rep] == list(range(nb)), "buckets issued out of order"
    queued = [ms for _, _, _, ms in rep]
    # all but the tail (the stem's gradients, complete at the very end) leave backward compute
    # behind them; the first bucket is issued in the first half of backward
    assert all(ms > 0.05 for ms in queued[:-1]), queued
    assert queued[0] > 0.5 * bwd_ms, (queued[0], bwd_ms)
    print(f"backward {bwd_ms:.2f} ms; compute queued behind each bucket issue (ms): "
          + ", ".join(f"{ms:.2f}" for ms in queued))
