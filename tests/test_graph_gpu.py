"""HIP-graph captured training step (deep_vision_amd/train/graph.py): replays must reproduce the
eager trajectory -- same parameters after N steps with SGD-momentum and with Adam (device-side LR /
bias correction), LR changes between replays honoured, BatchNorm batch counts advanced."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _net():
    from deep_vision_amd import nn

    torch.manual_seed(0)
    return torch.nn.Sequential(nn.Conv2d(8, 32, 3, padding=1, bias=False), nn.BatchNorm2d(32), nn.ReLU(),
                               nn.Conv2d(32, 16, 3, stride=2, padding=1), nn.AdaptiveAvgPool2d((1, 1)),
                               torch.nn.Flatten(), nn.Linear(16, 10)).to(DEV)


@pytest.mark.parametrize("opt_name", ["SGD", "Adam"])
def test_captured_step_matches_eager(opt_name):
    from deep_vision_amd import ops as F
    from deep_vision_amd.train.graph import CapturedStep
    from deep_vision_amd.train.optim import OPTIMIZERS

    kw = dict(lr=0.05, momentum=0.9, weight_decay=1e-4) if opt_name == "SGD" else dict(lr=1e-3)
    a = _net()
    b = copy.deepcopy(a)
    oa, ob = OPTIMIZERS[opt_name](a.parameters(), **kw), OPTIMIZERS[opt_name](b.parameters(), **kw)
    xs = [torch.randn(16, 8, 20, 20, device=DEV) for _ in range(8)]
    ys = [torch.randint(0, 10, (16,), device=DEV) for _ in range(8)]

    def make_step(model, opt):
        def step(x, y):
            opt.zero_grad()
            loss = F.cross_entropy(model(x), y)
            loss.backward()
            opt.step()
            return loss
        return step

    sa = make_step(a, oa)
    for i in range(8):  # eager reference: 8 steps, LR halved after step 5
        if i == 5:
            for g in oa.param_groups:
                g["lr"] *= 0.5
        sa(xs[i], ys[i])
    # captured: 2 eager warm-up steps on a side stream (the first two batches), then replays
    xst, yst = xs[0].clone(), ys[0].clone()
    it = iter(range(2))
    warm = [(xs[0], ys[0]), (xs[1], ys[1])]
    step_b = make_step(b, ob)

    def step_fn(x, y):
        k = next(it, None)
        if k is not None:  # the warm-up calls consume the first two batches
            x.copy_(warm[k][0]); y.copy_(warm[k][1])
        return step_fn.inner(x, y)

    step_fn.inner = step_b
    cap = CapturedStep(step_fn, ob, (xst, yst), model=b, warmup=2)
    for i in range(2, 8):
        if i == 5:
            for g in ob.param_groups:
                g["lr"] *= 0.5
        cap(xs[i], ys[i])
    torch.cuda.synchronize()
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        err = ((pa - pb).abs().max() / pa.abs().max().clamp_min(1e-6)).item()
        assert err < 1e-3, (n, err)
    assert ob._flat[0]["step"] == oa._flat[0]["step"] == 8
    assert int(b[1].state_dict()["num_batches_tracked"]) == int(a[1].state_dict()["num_batches_tracked"]) == 8


def test_classifier_trainer_graph_mode(tmp_path):
    """run_epochs(..., graph=True): the step is captured on the first batch and replayed; the
    short last batch of the epoch runs eagerly (a second signature would be captured, capped at 2)."""
    from deep_vision_amd.config import get_config
    from deep_vision_amd.train.classification import run_epochs

    cfg = get_config("lenet5")
    last, loggers = run_epochs(cfg, None, device="cuda", synthetic=True, synthetic_size=200, num_workers=0, epochs=1,
                               max_steps=4, val_steps=1, checkpoint_dir=str(tmp_path) + "/", graph=True)
    assert last
    assert all(v == v for v in loggers["train_loss"]["value"])  # finite (no NaN) losses


def test_hourglass_trainer_graph_mode(tmp_path):
    from deep_vision_amd.config import get_config
    from deep_vision_amd.train.detection import train

    cfg = get_config("hourglass", input_shape=(3, 64, 64), batch_size=2)
    cfg = cfg.replace(model_params={**cfg.model_params, "num_stack": 2})
    best = train(cfg, synthetic=True, synthetic_size=6, epochs=1, device="cuda", workers=0, log_every=1,
                 checkpoint_dir=str(tmp_path), tensorboard_dir=str(tmp_path / "tb"), graph=True)
    assert best


def test_two_signatures_share_device_hparams():
    """a second capture (short last batch) must not replace the device LR tensor
    the first graph baked in. Sequence: full, full, short (2nd capture), LR x0.1, full (replay of
    graph 1), short (replay of graph 2), full -- equal to the same steps run eagerly."""
    from deep_vision_amd import ops as F
    from deep_vision_amd.train.graph import GraphedTrainStep
    from deep_vision_amd.train.optim import OPTIMIZERS

    a = _net()
    b = copy.deepcopy(a)
    kw = dict(lr=1e-2, betas=(0.9, 0.999))
    oa, ob = OPTIMIZERS["Adam"](a.parameters(), **kw), OPTIMIZERS["Adam"](b.parameters(), **kw)
    sizes = [16, 16, 8, 16, 8, 16]
    xs = [torch.randn(n, 8, 20, 20, device=DEV) for n in sizes]
    ys = [torch.randint(0, 10, (n,), device=DEV) for n in sizes]

    def fl_a(x, y):
        return F.cross_entropy(a(x), y), None

    def fl_b(x, y):
        return F.cross_entropy(b(x), y), None

    def eager_a(x, y):
        oa.zero_grad()
        loss = fl_a(x, y)[0]
        loss.backward()
        oa.step()
        return loss, None

    gs = GraphedTrainStep(b, ob, fl_b, eager_step=None, max_graphs=2)
    for i in range(len(sizes)):
        if i == 3:
            for o in (oa, ob):
                for g in o.param_groups:
                    g["lr"] *= 0.1
        eager_a(xs[i], ys[i])
        gs(xs[i], ys[i])
    torch.cuda.synchronize()
    assert len(gs.graphs) == 2
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        err = ((pa - pb).abs().max() / pa.abs().max().clamp_min(1e-6)).item()
        assert err < 2e-3, (n, err)
    assert ob._flat[0]["step"] == oa._flat[0]["step"] == len(sizes)


def _graph_dp_worker(port, q):
    """World-1 RCCL group, DataParallel forced on: 10 eager DP steps vs 2 eager warm-up + 8 replays
    of the captured DP step (bucket all-reduces inside the graph)."""
    import os

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    from deep_vision_amd import nn, ops as F, set_deterministic
    from deep_vision_amd.parallel.ddp import DataParallel
    from deep_vision_amd.parallel.dist import init_distributed
    from deep_vision_amd.train.graph import CapturedStep, prepare_capture_env
    from deep_vision_amd.train.optim import FusedSGD

    prepare_capture_env()
    init_distributed("nccl", force=True)
    set_deterministic(True)

    def net():
        torch.manual_seed(0)
        return torch.nn.Sequential(nn.Conv2d(8, 64, 3, padding=1, bias=False), nn.ReLU(),
                                   nn.Conv2d(64, 64, 3, padding=1, bias=False), nn.ReLU(),
                                   nn.Conv2d(64, 16, 1, bias=False), nn.AdaptiveAvgPool2d((1, 1)),
                                   torch.nn.Flatten(), nn.Linear(16, 10, bias=False)).to(DEV)

    xs = [torch.randn(16, 8, 20, 20, device=DEV) for _ in range(10)]
    ys = [torch.randint(0, 10, (16,), device=DEV) for _ in range(10)]
    res = []
    for mode in ("eager", "graph"):
        m = net()
        ddp = DataParallel(m, bucket_mb=0.02, always_reduce=True)
        opt = FusedSGD(m.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
        xst, yst = xs[0].clone(), ys[0].clone()
        it = iter(range(2))

        def step(x, y):
            k = next(it, None) if mode == "graph" else None
            if k is not None:  # the warm-up calls consume the first two batches
                x.copy_(xs[k]); y.copy_(ys[k])
            opt.zero_grad()
            loss = F.cross_entropy(ddp(x), y)
            loss.backward()
            ddp.finish()
            opt.step(grad_scale=ddp.grad_scale)
            return loss

        if mode == "eager":
            for i in range(10):
                step(xs[i], ys[i])
        else:
            cap = CapturedStep(step, opt, (xst, yst), model=m, warmup=2)
            calls = ddp.comm_stats["allreduce_calls"]
            for i in range(2, 10):
                cap(xs[i], ys[i])
            assert ddp.comm_stats["allreduce_calls"] == calls  # replays run no Python hooks
        torch.cuda.synchronize()
        res.append(torch.cat([p.detach().reshape(-1).cpu() for p in m.parameters()]).numpy())
        nb = len(ddp.buckets)
    q.put((res, nb))
    import torch.distributed as dist

    dist.destroy_process_group()


def test_dp_step_captured_with_rccl_allreduce():
    """the DP step (bucketed RCCL all-reduce included) captured in a HIP graph
    replays the eager DP trajectory over 10 steps."""
    import torch.multiprocessing as mp

    from deep_vision_amd.launch import free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_graph_dp_worker, args=(free_port(), q))
    p.start()
    (eager, graph), nb = q.get(timeout=180)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert nb >= 2
    e, g = torch.from_numpy(eager), torch.from_numpy(graph)
    assert ((e - g).abs().max() / e.abs().max()).item() < 1e-5


def _nan_graph_worker(port, q):
    """World-1 RCCL group, DataParallel forced on, device non-finite guard: a captured DP step
    whose replay sees a NaN input batch leaves parameters, momentum and BN running statistics
    untouched, counts the skip on the device, and the next finite replay trains normally."""
    import os

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    from deep_vision_amd import nn, ops as F
    from deep_vision_amd.parallel.ddp import DataParallel
    from deep_vision_amd.parallel.dist import init_distributed
    from deep_vision_amd.train.graph import CapturedStep, prepare_capture_env
    from deep_vision_amd.train.optim import FusedSGD

    prepare_capture_env()
    init_distributed("nccl", force=True)
    torch.manual_seed(0)
    m = torch.nn.Sequential(nn.Conv2d(8, 32, 3, padding=1, bias=False), nn.BatchNorm2d(32), nn.ReLU(),
                            nn.AdaptiveAvgPool2d((1, 1)), torch.nn.Flatten(), nn.Linear(32, 10)).to(DEV)
    ddp = DataParallel(m, bucket_mb=0.01, always_reduce=True)
    opt = FusedSGD(m.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    opt.use_device_guard(True)
    xst = torch.randn(16, 8, 12, 12, device=DEV)
    yst = torch.randint(0, 10, (16,), device=DEV)

    def step(x, y):
        opt.zero_grad()
        loss = F.cross_entropy(ddp(x), y)
        loss.backward()
        ddp.finish()
        opt.step(grad_scale=ddp.grad_scale)
        return loss

    cap = CapturedStep(step, opt, (xst, yst), model=m, warmup=2)
    cap(torch.randn(16, 8, 12, 12, device=DEV), yst)
    torch.cuda.synchronize()
    snap = lambda: (opt._flat[0]["param"].clone(), opt._flat[0]["states"]["momentum_buffer"].clone(),  # noqa: E731
                    m[1].running_mean.clone(), m[1].running_var.clone())
    before = snap()
    bad = torch.randn(16, 8, 12, 12, device=DEV)
    bad[3, 2, 5, 5] = float("nan")
    cap(bad, yst)
    torch.cuda.synchronize()
    after = snap()
    skipped_ok = all(torch.equal(a, b) for a, b in zip(before, after))
    c1 = opt.device_guard_counts()
    cap(torch.randn(16, 8, 12, 12, device=DEV), yst)
    torch.cuda.synchronize()
    moved = not torch.equal(opt._flat[0]["param"], before[0])
    finite = bool(torch.isfinite(opt._flat[0]["param"]).all())
    q.put((skipped_ok, c1, opt.device_guard_counts(), moved, finite))
    import torch.distributed as dist

    dist.destroy_process_group()


def test_captured_dp_step_skips_nonfinite_on_device():
    """the NaN skip works inside the graph-captured DP step."""
    import torch.multiprocessing as mp

    from deep_vision_amd.launch import free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nan_graph_worker, args=(free_port(), q))
    p.start()
    skipped_ok, c1, c2, moved, finite = q.get(timeout=180)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert skipped_ok, "a non-finite replay changed parameters / optimizer state / BN running stats"
    assert c1 == (1, 1, True)
    assert c2 == (1, 0, False)
    assert moved and finite


def test_captured_dropout_draws_fresh_masks_per_replay():
    """A captured step bakes each dropout call's host seed into the graph; the per-device step
    counter (ops/act.py, advanced by CapturedStep before each replay) still gives every replay its
    own masks, and the backward reuses its forward's mask."""
    from deep_vision_amd import nn, ops as F
    from deep_vision_amd.train.graph import CapturedStep
    from deep_vision_amd.train.optim import FusedSGD

    torch.manual_seed(0)
    lin = nn.Linear(64, 64).to(DEV)
    opt = FusedSGD(lin.parameters(), lr=0.0)
    x = torch.randn(32, 64, device=DEV)
    outs = []

    def step(xx):
        opt.zero_grad()
        y = F.dropout(lin(xx), 0.5, True)
        y.float().sum().backward()
        opt.step()
        return y.detach().float().clone(), lin.weight.grad.detach().clone()

    cap = CapturedStep(step, opt, (x,), model=lin, warmup=1)
    for _ in range(3):
        y, g = cap(x)
        outs.append((y.clone(), g.clone()))
    torch.cuda.synchronize()
    (y0, g0), (y1, g1) = outs[0], outs[1]
    assert not torch.equal(y0 != 0, y1 != 0), "replays reused the captured dropout mask"
    assert 0.4 < (y0 != 0).float().mean().item() < 0.6
    # the weight gradient is sum over kept outputs of x: consistent with the forward's mask
    keep = (y1 != 0).float() * 2.0
    ref = keep.t() @ x
    assert torch.allclose(g1, ref, rtol=2e-2, atol=2e-1)


def test_engine_graph_step_with_comm_watchdog():
    """Engine.train_step(graph=True) with a comm watchdog attached (as on a multi-rank job): the
    capture records no watched event (an event recorded in a capture cannot be queried) and the
    watchdog does not poll while the capture runs; the replays are tracked and complete."""
    from deep_vision_amd import ops as F
    from deep_vision_amd.parallel.watchdog import CommWatchdog
    from deep_vision_amd.train.engine import Engine
    from deep_vision_amd.train.optim import FusedSGD

    eng = Engine(device="cuda", graph=True)
    fired = []
    eng.comm_watchdog = CommWatchdog(timeout=60, poll=0.01, on_timeout=lambda c, why: fired.append((c, why))).start()
    try:
        model = _net()
        opt = FusedSGD(model.parameters(), lr=0.01, momentum=0.9)
        x = torch.randn(16, 8, 20, 20, device=DEV)
        y = torch.randint(0, 10, (16,), device=DEV)

        def fl(xx, yy):
            return F.cross_entropy(model(xx), yy), None

        losses = [eng.train_step(model, opt, fl, x, y)[0].item() for _ in range(5)]
        torch.cuda.synchronize()
        import time

        time.sleep(0.2)  # a few polls after the last replay
        assert not fired, fired
        assert all(v == v for v in losses)
        assert eng.comm_watchdog.pending() <= 1
    finally:
        eng.comm_watchdog.stop()


def test_captured_adam_skipped_step_keeps_bias_correction():
    """a replay the device guard skips must not advance Adam's bias corrections (an eager
    skipped step never calls step()). Captured run: warm-up, replay(x1), replay(NaN batch),
    replay(x3); it must match eager steps on the same batches without the NaN one, and differ
    from a run whose step count did advance over the skip."""
    from deep_vision_amd import nn
    from deep_vision_amd.train.graph import CapturedStep
    from deep_vision_amd.train.optim import FusedAdam

    torch.manual_seed(0)
    base = nn.Linear(32, 16).to(DEV)
    xs = [torch.randn(64, 32, device=DEV) for _ in range(3)]
    bad = xs[1].clone()
    bad[5, 3] = float("nan")

    def make():
        m = copy.deepcopy(base)
        return m, FusedAdam(m.parameters(), lr=1e-2, betas=(0.9, 0.999))

    def step_fn(m, opt):
        def step(x):
            opt.zero_grad()
            loss = (m(x).float() ** 2).mean()
            loss.backward()
            opt.step()
            return loss
        return step

    m, opt = make()
    opt.use_device_guard(True)
    cap = CapturedStep(step_fn(m, opt), opt, (xs[0].clone(),), model=m, warmup=2)
    for x in (xs[0], bad, xs[2]):
        cap(x)
    torch.cuda.synchronize()
    assert opt.device_guard_counts()[0] == 1
    got = torch.cat([p.detach().flatten() for p in m.parameters()])

    def eager(skip_advances):
        me, oe = make()
        st = step_fn(me, oe)
        for x in (xs[0], xs[0], xs[0]):  # the two warm-up steps, then replay 1
            st(x)
        if skip_advances:
            for f in oe._flat:
                if f is not None:
                    f["step"] += 1
        st(xs[2])
        torch.cuda.synchronize()
        return torch.cat([p.detach().flatten() for p in me.parameters()])

    ref, wrong = eager(False), eager(True)
    rel = lambda a, b: ((a - b).norm() / b.norm()).item()  # noqa: E731
    assert rel(got, ref) < 1e-4, (rel(got, ref), rel(got, wrong))
    assert rel(wrong, ref) > 10 * rel(got, ref)
