"""Stacked Hourglass branch concurrency (models/hourglass.py BRANCH_STREAMS): each level's up1
branch on a side stream gives the same step as the single-stream run, eagerly and as a captured
HIP graph whose replays follow the eager trajectory."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _net():
    from deep_vision_amd.models.hourglass import StackedHourglassNetwork

    torch.manual_seed(0)
    return StackedHourglassNetwork(num_stack=2, num_residual=1, num_heatmap=16).to(DEV)


def _loss(ys, hm):
    from deep_vision_amd.ops.loss import heatmap_mse

    return sum(heatmap_mse(y, hm) for y in ys)


def _grads(m):
    return torch.cat([p.grad.detach().float().reshape(-1) for p in m.parameters() if p.grad is not None])


def _params(m):
    return torch.cat([p.detach().float().reshape(-1) for p in m.parameters()])


def test_branch_streams_match_single_stream():
    """Deterministic mode: forking the up1 branches onto side streams changes no arithmetic -- the
    single-stream and the forked forward + backward give bitwise-equal loss and gradients, run after
    run (a cross-stream ordering bug would show as a difference here)."""
    from deep_vision_amd import set_deterministic
    from deep_vision_amd.models import hourglass as H

    x = torch.randn(4, 3, 128, 128, device=DEV)
    hm = torch.rand(4, 16, 32, 32, device=DEV)
    base = _net()
    res = []
    saved = H.BRANCH_STREAMS
    set_deterministic(True)
    try:
        for on in (False, False, True, True):
            H.BRANCH_STREAMS = on
            m = copy.deepcopy(base)
            loss = _loss(m(x), hm)
            loss.backward()
            torch.cuda.synchronize()
            res.append((loss.detach().float().clone(), _grads(m)))
    finally:
        H.BRANCH_STREAMS = saved
        set_deterministic(False)
    assert len(H._STREAMS) >= 1
    for k in range(1, 4):
        assert torch.equal(res[0][0], res[k][0]), (k, res[0][0].item(), res[k][0].item())
        assert torch.equal(res[0][1], res[k][1]), (k, (res[0][1] - res[k][1]).abs().max().item())


def test_side_stream_wgrad_with_optout_disabled_matches_origin_stream():
    """with the Hourglass no_wgrad_side opt-out ignored (what DV_WGRAD_SIDE_OPTOUT=0
    does), weight gradients run on the side stream. A residual-epilogue conv hands its dy on to a BN
    backward that overwrites it in place on the origin stream, so such convs must keep their weight
    gradient on the origin stream; deterministic mode, so the side-stream step must equal the
    all-origin step bitwise."""
    from deep_vision_amd import set_deterministic
    from deep_vision_amd.models import hourglass as H
    from deep_vision_amd.ops import conv as C

    x = torch.randn(4, 3, 128, 128, device=DEV)
    hm = torch.rand(4, 16, 32, 32, device=DEV)
    base = _net()
    res = []
    saved = (C._SIDE_OPTOUT, C.WGRAD_SIDE, H.BRANCH_STREAMS)
    set_deterministic(True)
    try:
        H.BRANCH_STREAMS = False
        for side in (False, True, True):
            C._SIDE_OPTOUT = not side
            C.WGRAD_SIDE = saved[1] if side else 0
            m = copy.deepcopy(base)
            loss = _loss(m(x), hm)
            loss.backward()
            C.wgrad_side_join()
            torch.cuda.synchronize()
            res.append((loss.detach().float().clone(), _grads(m)))
    finally:
        C._SIDE_OPTOUT, C.WGRAD_SIDE, H.BRANCH_STREAMS = saved
        set_deterministic(False)
    for k in (1, 2):
        assert torch.equal(res[0][0], res[k][0])
        assert torch.equal(res[0][1], res[k][1]), (k, (res[0][1] - res[k][1]).abs().max().item())


def _six_steps(base, xs, hms, captured, lr=1e-4):
    """6 SGD steps: eagerly on one stream, or as a captured step (2 eager warm-up steps on the capture
    stream consume the first two batches, then 4 replays) with the up1 branches forked."""
    from deep_vision_amd.models import hourglass as H
    from deep_vision_amd.train.graph import CapturedStep
    from deep_vision_amd.train.optim import FusedSGD

    m = copy.deepcopy(base)
    o = FusedSGD(m.parameters(), lr=lr)

    def step(x, hm):
        o.zero_grad()
        loss = _loss(m(x), hm)
        loss.backward()
        o.step()
        return loss

    if not captured:
        saved = H.BRANCH_STREAMS
        H.BRANCH_STREAMS = False
        try:
            losses = [step(xs[i], hms[i]).detach().float().clone() for i in range(6)]
        finally:
            H.BRANCH_STREAMS = saved
        torch.cuda.synchronize()
        return torch.stack(losses), _params(m)
    assert H.BRANCH_STREAMS in ("graph", True)
    warm = iter([(xs[0], hms[0]), (xs[1], hms[1])])

    def step_fn(x, hm):
        w = next(warm, None)
        if w is not None:
            x.copy_(w[0])
            hm.copy_(w[1])
        return step(x, hm)

    cap = CapturedStep(step_fn, o, (xs[0].clone(), hms[0].clone()), model=m, warmup=2)
    losses = [cap.warmup_outputs.detach().float().clone()]
    losses += [cap(xs[i], hms[i]).detach().float().clone() for i in range(2, 6)]
    torch.cuda.synchronize()
    assert 4 in H._FORKED, "capture did not fork the up1 branches"
    assert len({k[1] for k in H._STREAMS}) <= H.side_streams()
    return torch.stack(losses), _params(m)


def test_branch_streams_captured_step_matches_eager():
    """Deterministic mode: the captured, branch-forked step replays the eager single-stream
    trajectory bit for bit over 6 SGD steps (losses from step 1 on, and the final weights)."""
    from deep_vision_amd import set_deterministic

    xs = [torch.randn(4, 3, 128, 128, device=DEV) for _ in range(6)]
    hms = [torch.rand(4, 16, 32, 32, device=DEV) for _ in range(6)]
    base = _net()
    set_deterministic(True)
    try:
        le, pe = _six_steps(base, xs, hms, captured=False)
        lc, pc = _six_steps(base, xs, hms, captured=True)
    finally:
        set_deterministic(False)
    print("eager", le.tolist(), "captured (from step 1)", lc.tolist())
    assert torch.equal(le[1:], lc), (le.tolist(), lc.tolist())
    assert torch.equal(pe, pc), (pe - pc).abs().max().item()


def test_branch_streams_captured_step_tolerance_default_mode():
    """Default (atomic) mode at a well-conditioned size (batch 16, 256x256 input: the deepest level
    is 4x4, 256 values per BN channel): the captured forked step trains like the eager one over 6
    steps. Exactness is the deterministic test above; in the default mode a random-init network
    turns summation-order rounding into O(1e-3) trajectory differences (measured: losses within
    1.0e-3 relative, weights within 2.4e-3 -- tools/diag_noise.py shows the same sensitivity to a
    1e-6 input perturbation), so this bounds a broken capture (wrong stream joins, stale scratch),
    not rounding."""
    torch.manual_seed(1)
    xs = [torch.randn(16, 3, 256, 256, device=DEV) for _ in range(6)]
    hms = [torch.rand(16, 16, 64, 64, device=DEV) for _ in range(6)]
    base = _net()
    le, pe = _six_steps(base, xs, hms, captured=False)
    lc, pc = _six_steps(base, xs, hms, captured=True)
    print("eager", le.tolist(), "captured (from step 1)", lc.tolist())
    rel = ((le[1:] - lc).abs() / le[1:].abs()).max().item()
    drift = ((pe - pc).norm() / pe.norm()).item()
    print("max relative loss difference", rel, "relative weight drift", drift)
    assert (lc[1:] < lc[:-1]).all(), lc.tolist()  # it trains
    assert rel < 1e-2, rel
    assert drift < 2e-2, drift


def test_block_statistics_handoff_matches_separate_pass():
    """BottleneckBlock conv3 epilogues accumulating the next block's pre-activation BN statistics
    (post-residual, csrc/conv_fwd_core.h RST) give the forward / backward of the separate
    statistics pass: two chained blocks (shallow enough that rounding differences stay
    rounding-sized), batch statistics, running statistics and gradients compared."""
    from deep_vision_amd.models import hourglass as H

    torch.manual_seed(0)
    blocks = torch.nn.Sequential(H.BottleneckBlock(128, 128), H.BottleneckBlock(128, 128)).to(DEV)
    x32 = torch.randn(8, 128, 24, 24, device=DEV) * 2 + 0.5
    res = {}
    try:
        for on in (False, True):
            H.HANDOFF_STATS = on
            m = copy.deepcopy(blocks)
            x = x32.to(torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_(True)
            y = H._run_blocks(m, x)
            g = torch.randn(y.shape, device=DEV, generator=torch.Generator(device=DEV).manual_seed(1))
            y.backward(g.to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
            torch.cuda.synchronize()
            res[on] = (y.detach().float(), x.grad.float(), _grads(m), m[1].bn1.running_mean.clone(),
                       m[1].bn1.running_var.clone())
    finally:
        H.HANDOFF_STATS = True
    (y0, dx0, g0, rm0, rv0), (y1, dx1, g1, rm1, rv1) = res[False], res[True]
    assert torch.allclose(rm0, rm1, rtol=1e-3, atol=1e-4) and torch.allclose(rv0, rv1, rtol=1e-3, atol=1e-4)
    assert ((y0 - y1).norm() / y0.norm()).item() < 1e-2
    cos = lambda a, b: torch.nn.functional.cosine_similarity(a.flatten(), b.flatten(), dim=0).item()
    assert cos(dx0, dx1) > 0.999 and cos(g0, g1) > 0.999
    assert not any("_dv_block_stats" in b.__dict__ for b in blocks.modules())


@pytest.mark.parametrize("forked", [False, True])
def test_level_gradient_join_matches_autograd_adds(forked):
    """An hourglass level input's three gradients (block 0's BN1, its identity shortcut, the pooled
    low branch) summed in block 0's BN1 backward apply pass (models/hourglass.py LEVEL_JOIN) give
    the autograd-add gradients -- single stream, and with up1 on a side stream (the pooled
    gradient then crosses streams through the join)."""
    from deep_vision_amd.models import hourglass as H
    from deep_vision_amd.ops.bn import COUNTERS

    torch.manual_seed(0)
    level = H.HourglassModule(2, 128, 1).to(DEV)
    x32 = torch.randn(8, 128, 16, 16, device=DEV)
    res = {}
    saved = H.BRANCH_STREAMS
    try:
        H.BRANCH_STREAMS = forked
        for on in (False, True):
            H.LEVEL_JOIN = on
            m = copy.deepcopy(level)
            x = x32.to(torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_(True)
            n0 = COUNTERS["bwd_apply_two_addends"]
            y = m(x)
            g = torch.randn(y.shape, device=DEV, generator=torch.Generator(device=DEV).manual_seed(1))
            y.backward(g.to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
            torch.cuda.synchronize()
            res[on] = (y.detach().float(), x.grad.float(), _grads(m), COUNTERS["bwd_apply_two_addends"] - n0)
    finally:
        H.LEVEL_JOIN = True
        H.BRANCH_STREAMS = saved
    (y0, dx0, g0, n_off), (y1, dx1, g1, n_on) = res[False], res[True]
    assert n_off == 0 and n_on == 2, (n_off, n_on)  # both levels folded their pooled gradient
    assert torch.equal(y0, y1)
    rel = lambda a, b: ((a - b).norm() / a.norm()).item()  # noqa: E731
    assert rel(dx0, dx1) < 1e-2, rel(dx0, dx1)
    assert rel(g0, g1) < 1e-2, rel(g0, g1)


def test_bias_gradient_from_bn_backward_matches_reduction_pass():
    """conv3's bias gradient folded from the next block's BN1 backward apply pass (the pass sums
    the gradient it writes, csrc/bn.hip bn_bwd_apply colsum; models/hourglass.py BIAS_COLSUM) equals
    the separate per-channel reduction of that gradient; every other gradient is unchanged."""
    from deep_vision_amd.models import hourglass as H
    from deep_vision_amd.ops.conv import COUNTERS_BIAS

    torch.manual_seed(0)
    blocks = torch.nn.Sequential(*[H.BottleneckBlock(128, 128) for _ in range(3)]).to(DEV)
    x32 = torch.randn(8, 128, 24, 24, device=DEV)
    res = {}
    try:
        for on in (False, True):
            H.BIAS_COLSUM = on
            m = copy.deepcopy(blocks)
            x = x32.to(torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_(True)
            n0 = COUNTERS_BIAS["colsum_fused"]
            y = H._run_blocks(m, x)
            g = torch.randn(y.shape, device=DEV, generator=torch.Generator(device=DEV).manual_seed(1))
            y.backward(g.to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
            torch.cuda.synchronize()
            res[on] = ([p.grad.float().clone() for p in m.parameters()], x.grad.float(),
                       COUNTERS_BIAS["colsum_fused"] - n0)
    finally:
        H.BIAS_COLSUM = True
    (g0, dx0, n_off), (g1, dx1, n_on) = res[False], res[True]
    assert n_off == 0 and n_on == 2, (n_off, n_on)  # blocks 0 and 1 hand their bias gradient over
    assert torch.equal(dx0, dx1)
    for i, (a, b) in enumerate(zip(g0, g1)):
        rel = ((a - b).norm() / a.norm().clamp_min(1e-12)).item()
        assert rel < 1e-3, (i, rel)


@pytest.mark.parametrize("op", ["maxpool", "upsample_add"])
def test_pool_fused_bn_statistics(op):
    """max pool / upsample-add passes accumulating the consumer BN's statistics of their output
    (csrc/pool.hip PoolStats): the shard sums equal the fp32 per-channel sum and sum of squares of
    the stored output (shift row zero)."""
    from deep_vision_amd import ops as F
    from deep_vision_amd.ops.bn import STAT_ROWS, STAT_SHARDS

    g = torch.Generator(device=DEV).manual_seed(4)
    x = torch.randn(8, 256, 32, 32, device=DEV, generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    buf = torch.zeros((STAT_ROWS, 256), device=DEV)
    if op == "maxpool":
        y, st = F.max_pool2d(x, 2, 2, stats_buf=buf)
        ref = torch.nn.functional.max_pool2d(x.float(), 2, 2)
    else:
        low = torch.randn(8, 256, 16, 16, device=DEV, generator=g).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        y, st = F.upsample_add(low, x, 2, stats_buf=buf)
        ref = (torch.nn.functional.interpolate(low.float(), scale_factor=2, mode="nearest") + x.float())
    torch.cuda.synchronize()
    assert st is not None
    assert torch.allclose(y.float(), ref.to(torch.bfloat16).float())
    sh = buf[: 2 * STAT_SHARDS].view(STAT_SHARDS, 2, 256).sum(0)
    yf = y.float()
    s_ref, q_ref = yf.sum((0, 2, 3)), (yf * yf).sum((0, 2, 3))
    assert torch.allclose(sh[0], s_ref, rtol=1e-4, atol=1e-2), (sh[0] - s_ref).abs().max().item()
    assert torch.allclose(sh[1], q_ref, rtol=1e-4, atol=1e-2), (sh[1] - q_ref).abs().max().item()


def test_level_statistics_handoff_matches_separate_passes():
    """A whole hourglass level with every pre-activation BN statistic handed over (conv3 epilogues,
    the pool and the merge pass) trains like the level with separate statistics passes."""
    from deep_vision_amd.models import hourglass as H

    torch.manual_seed(0)
    level = H.HourglassModule(2, 128, 1).to(DEV)
    nxt = H.BottleneckBlock(128, 128).to(DEV)
    x32 = torch.randn(8, 128, 16, 16, device=DEV) * 2 + 0.5
    res = {}
    try:
        for on in (False, True):
            H.HANDOFF_STATS = on
            m, b = copy.deepcopy(level), copy.deepcopy(nxt)
            x = x32.to(torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_(True)
            y = H._run_blocks([b], m(x, next_bn=b.bn1))
            g = torch.randn(y.shape, device=DEV, generator=torch.Generator(device=DEV).manual_seed(1))
            y.backward(g.to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
            torch.cuda.synchronize()
            res[on] = (y.detach().float(), x.grad.float(), _grads(m), torch.cat([bf.float().flatten() for bf in m.buffers() if bf.is_floating_point()]),
                       b.bn1.running_mean.clone())
    finally:
        H.HANDOFF_STATS = True
    (y0, dx0, g0, b0, r0), (y1, dx1, g1, b1, r1) = res[False], res[True]
    assert torch.allclose(r0, r1, rtol=1e-3, atol=1e-4)
    assert ((b0 - b1).norm() / b0.norm()).item() < 1e-4
    assert ((y0 - y1).norm() / y0.norm()).item() < 1e-2
    cos = lambda a, b: torch.nn.functional.cosine_similarity(a.flatten(), b.flatten(), dim=0).item()  # noqa: E731
    assert cos(dx0, dx1) > 0.999 and cos(g0, g1) > 0.999
    assert not any("_dv_block_stats" in mm.__dict__ for mm in list(m.modules()) + list(b.modules()))

