"""Depthwise conv kernels (csrc/depthwise.hip) beyond the basic shapes of test_ops_gpu.py
(ADVICE r1): fused bias / activation / BatchNorm-statistics epilogues, a partial last channel
slab (C = 1040) with statistics, Keras asymmetric 'same' padding at stride 2 (mobilenet1_tf),
bitwise-deterministic weight gradients, and a MobileNet production shape (batch 128, 112x112)
-- all against a plain PyTorch fp32 reference of the same op."""
import pytest
import torch
import torch.nn.functional as TF

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def _nhwc(t):
    return t.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


def _ref_act(y, act):
    if act == "relu":
        return TF.relu(y)
    if act == "leaky":
        return TF.leaky_relu(y, 0.1)
    return y


@pytest.mark.parametrize("C,s", [(64, 1), (64, 2), (1040, 1), (1040, 2)])
@pytest.mark.parametrize("bias", [False, True])
@pytest.mark.parametrize("act", [None, "relu", "leaky"])
def test_depthwise_epilogue_and_stats(C, s, bias, act):
    from deep_vision_amd import ops as F

    torch.manual_seed(C + s)
    x32 = torch.randn(2, C, 14, 14, device=DEV).bfloat16().float()
    w = (torch.randn(C, 1, 3, 3, device=DEV) * 0.3).requires_grad_(True)
    b = (torch.randn(C, device=DEV) * 0.5).requires_grad_(True) if bias else None
    x = _nhwc(x32).requires_grad_(True)
    y, stats = F.conv2d(x, w, b, s, 1, 1, C, act=act, slope=0.1, want_stats=True)
    xr = x32.clone().requires_grad_(True)
    wr = w.detach().clone().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True) if bias else None
    yr = _ref_act(TF.conv2d(xr, wr, br, s, 1, 1, C), act)
    assert y.shape == yr.shape
    assert _rel(y, yr) < 2e-2
    # statistics of the fp32 outputs (before bf16 rounding), summed over the shards; a fresh
    # buffer's shift row (csrc/kernels.h DV_STAT_ROWS) is zero, so these are the plain sums
    yq = y.float()
    from deep_vision_amd.ops.bn import STAT_ROWS

    assert stats.shape[0] == STAT_ROWS and not stats[128:].any()  # shift row and ticket row
    tot = stats[:128].reshape(64, 2, -1).sum(0)
    assert _rel(tot[0, :C], yq.sum((0, 2, 3))) < 5e-3
    assert _rel(tot[1, :C], (yq * yq).sum((0, 2, 3))) < 5e-3
    dy = torch.randn_like(yr).bfloat16().float()
    y.backward(_nhwc(dy))
    yr.backward(dy)
    assert _rel(x.grad, xr.grad) < 3e-2
    assert _rel(w.grad, wr.grad) < 3e-2
    if bias:
        assert _rel(b.grad, br.grad) < 3e-2


@pytest.mark.parametrize("HW", [14, 15])
def test_depthwise_keras_same_stride2(HW):
    """padding (top, bottom, left, right) = Keras 'same' at stride 2: the extra bottom/right row
    is read as zeros by the gather (no padded copy)."""
    from deep_vision_amd import ops as F

    C, k, s = 64, 3, 2
    pt = max(k - s, 0) if HW % s == 0 else max(k - HW % s, 0)
    pad = (pt // 2, pt - pt // 2, pt // 2, pt - pt // 2)
    x32 = torch.randn(2, C, HW, HW, device=DEV).bfloat16().float()
    w = (torch.randn(C, 1, k, k, device=DEV) * 0.3).requires_grad_(True)
    x = _nhwc(x32).requires_grad_(True)
    y = F.conv2d(x, w, None, s, pad, 1, C)
    xr = x32.clone().requires_grad_(True)
    wr = w.detach().clone().requires_grad_(True)
    yr = TF.conv2d(TF.pad(xr, (pad[2], pad[3], pad[0], pad[1])), wr, None, s, 0, 1, C)
    assert y.shape == yr.shape == (2, C, -(-HW // s), -(-HW // s))
    assert _rel(y, yr) < 2e-2
    dy = torch.randn_like(yr).bfloat16().float()
    y.backward(_nhwc(dy))
    yr.backward(dy)
    assert _rel(x.grad, xr.grad) < 3e-2
    assert _rel(w.grad, wr.grad) < 3e-2


def test_depthwise_unsupported_stride_routes_grouped():
    """Stride (2, 1) is not a depthwise-kernel shape: it must take the grouped path and
    differentiate (round 1 failed in backward with 'dw_dgrad: unsupported shape')."""
    from deep_vision_amd import ops as F

    C = 64
    x32 = torch.randn(2, C, 12, 12, device=DEV).bfloat16().float()
    w = (torch.randn(C, 1, 3, 3, device=DEV) * 0.3).requires_grad_(True)
    x = _nhwc(x32).requires_grad_(True)
    y = F.conv2d(x, w, None, (2, 1), 1, 1, C)
    xr = x32.clone().requires_grad_(True)
    wr = w.detach().bfloat16().float().requires_grad_(True)
    yr = TF.conv2d(xr, wr, None, (2, 1), 1, 1, C)
    assert _rel(y, yr) < 2e-2
    dy = torch.randn_like(yr).bfloat16().float()
    y.backward(_nhwc(dy))
    yr.backward(dy)
    assert _rel(x.grad, xr.grad) < 3e-2
    assert _rel(w.grad, wr.grad) < 3e-2


def test_depthwise_wgrad_deterministic_bitwise():
    import deep_vision_amd as dv
    from deep_vision_amd import ops as F

    C = 256
    x = _nhwc(torch.randn(32, C, 28, 28, device=DEV))
    w = (torch.randn(C, 1, 3, 3, device=DEV) * 0.3).requires_grad_(True)
    dy = _nhwc(torch.randn(32, C, 28, 28, device=DEV))
    grads = []
    try:
        dv.set_deterministic(True)
        for _ in range(3):
            w.grad = None
            F.conv2d(x, w, None, 1, 1, 1, C).backward(dy)
            grads.append(w.grad.clone())
    finally:
        dv.set_deterministic(False)
    assert torch.equal(grads[0], grads[1]) and torch.equal(grads[1], grads[2])
    w.grad = None
    F.conv2d(x, w, None, 1, 1, 1, C).backward(dy)
    assert _rel(w.grad, grads[0]) < 1e-5


@pytest.mark.parametrize("C,HW,s", [(32, 112, 1), (64, 112, 2)])
def test_depthwise_mobilenet_production_shape(C, HW, s):
    """MobileNet V1's first depthwise layers at batch 128 (the bench config) vs fp32 torch."""
    from deep_vision_amd import ops as F

    N = 128
    x32 = torch.randn(N, C, HW, HW, device=DEV).bfloat16().float()
    w = (torch.randn(C, 1, 3, 3, device=DEV) * 0.3).requires_grad_(True)
    x = _nhwc(x32).requires_grad_(True)
    y = F.conv2d(x, w, None, s, 1, 1, C)
    xr = x32.clone().requires_grad_(True)
    wr = w.detach().clone().requires_grad_(True)
    yr = TF.conv2d(xr, wr, None, s, 1, 1, C)
    assert _rel(y, yr) < 2e-2
    dy = torch.randn_like(yr).bfloat16().float()
    y.backward(_nhwc(dy))
    yr.backward(dy)
    assert _rel(x.grad, xr.grad) < 3e-2
    assert _rel(w.grad, wr.grad) < 2e-2


@pytest.mark.parametrize("s,act", [(1, "relu"), (2, "relu"), (1, None), (2, "leaky")])
def test_depthwise_dgrad_fuses_bn_backward(s, act):
    """pw conv -> BN -> act -> dw conv (MobileNet block): the BN's backward reduction runs in the
    depthwise dgrad epilogue (csrc/depthwise.hip DwBnr) instead of a bn_bwd_reduce pass. The
    gradients equal the unfused native chain (same bf16 tensors, tight) and the fp32 torch chain
    (loose: ReLU masks of bf16 vs fp32 pre-activations differ near zero)."""
    from deep_vision_amd import nn
    from deep_vision_amd import ops as F
    from deep_vision_amd.ops import bn as B

    torch.manual_seed(7 + s)
    C = 64
    pw = nn.Conv2d(32, C, 1, bias=False).to(DEV)
    bn = nn.BatchNorm2d(C).to(DEV)
    dw = nn.Conv2d(C, C, 3, stride=s, padding=1, groups=C, bias=False).to(DEV)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    x32 = torch.randn(4, 32, 28, 28, device=DEV).bfloat16().float()
    dy = None

    def run(fuse):
        nonlocal dy
        B.FUSE_BWD_STATS = fuse
        try:
            for p in (pw.weight, bn.weight, bn.bias, dw.weight):
                p.grad = None
            x = _nhwc(x32).requires_grad_(True)
            n0 = B.COUNTERS["bwd_reduce_fused"]
            y = dw(F.conv_bn_act(x, pw, bn, act, slope=0.1))
            if dy is None:
                dy = torch.randn(y.shape, device=DEV).bfloat16().float()
            y.backward(_nhwc(dy))
            return (B.COUNTERS["bwd_reduce_fused"] - n0, y.float(), x.grad.float(), pw.weight.grad.clone(),
                    bn.weight.grad.clone(), bn.bias.grad.clone(), dw.weight.grad.clone())
        finally:
            B.FUSE_BWD_STATS = True

    fused = run(True)
    plain = run(False)
    # stride 1 folds the reduction into the dgrad epilogue; stride 2 keeps the reduce pass (and the
    # fused stride-2 kernel stays exercised through the binding below)
    assert fused[0] == (1 if s == 1 else 0) and plain[0] == 0, "BN reduction not fused into the depthwise dgrad"
    for a, b in zip(fused[1:], plain[1:]):
        assert _rel(a, b) < 2e-3
    ref = torch.nn.Sequential(torch.nn.Conv2d(32, C, 1, bias=False), torch.nn.BatchNorm2d(C),
                              torch.nn.ReLU() if act == "relu" else (torch.nn.LeakyReLU(0.1) if act else torch.nn.Identity()),
                              torch.nn.Conv2d(C, C, 3, stride=s, padding=1, groups=C, bias=False)).to(DEV)
    with torch.no_grad():
        ref[0].weight.copy_(pw.weight.bfloat16().float())
        ref[1].weight.copy_(bn.weight)
        ref[1].bias.copy_(bn.bias)
        ref[3].weight.copy_(dw.weight)
    xr = x32.clone().requires_grad_(True)
    yr = ref(xr)
    yr.backward(dy)
    def nrel(a, b):  # norm-relative: a few flipped ReLU masks move single elements, not the norm
        return ((a.float() - b.float()).norm() / b.float().norm()).item()

    assert nrel(fused[1], yr) < 2e-2
    assert nrel(fused[2], xr.grad) < 3e-2
    assert nrel(fused[4], ref[1].weight.grad) < 3e-2
    assert nrel(fused[5], ref[1].bias.grad) < 3e-2


@pytest.mark.parametrize("C,H,W,act,s", [(32, 112, 112, "relu", 1), (96, 13, 20, None, 1), (128, 9, 33, "leaky", 1),
                                         (512, 14, 14, "relu", 1), (64, 5, 70, None, 1),
                                         (64, 112, 112, "relu", 2), (96, 13, 20, None, 2), (128, 9, 33, "leaky", 2),
                                         (256, 28, 28, "relu", 2), (512, 14, 14, "relu", 2), (64, 5, 70, None, 2)])
def test_depthwise_tiled_matches_strip(C, H, W, act, s):
    """The LDS-tiled kernels (csrc/depthwise.hip dw_tile_kernel / dw_tile_wgrad_kernel; stride 2 with
    the even / odd split halo) against the strip kernels (benchmark variant 61) on ragged tiles:
    partial column / row tiles, several row bands per block, a 32-channel-multiple slab (C = 96),
    odd maps, with bias, activation and BN statistics. The forward and data gradient sum the taps
    in the same order (bitwise equal); the weight gradient and the statistics reduce in another
    order (fp32 rounding only)."""
    from deep_vision_amd import ops as F
    from deep_vision_amd._ext import lib

    torch.manual_seed(C + H + W)
    x32 = torch.randn(3, C, H, W, device=DEV).bfloat16().float()
    w0 = torch.randn(C, 1, 3, 3, device=DEV) * 0.3
    b0 = torch.randn(C, device=DEV) * 0.5
    P, Q = (H - 1) // s + 1, (W - 1) // s + 1
    dy = _nhwc(torch.randn(3, C, P, Q, device=DEV))

    def run(variant):
        lib().dw_variant(variant)
        try:
            x = _nhwc(x32).requires_grad_(True)
            w = w0.clone().requires_grad_(True)
            b = b0.clone().requires_grad_(True)
            y, stats = F.conv2d(x, w, b, s, 1, 1, C, act=act, slope=0.1, want_stats=True)
            y.backward(dy)
            torch.cuda.synchronize()
            return y.detach(), stats[:128].reshape(64, 2, -1).sum(0)[:, :C], x.grad, w.grad, b.grad
        finally:
            lib().dw_variant(0)

    tiled, strip = run(60), run(61)  # LDS tiles everywhere vs strip / plane kernels everywhere
    assert torch.equal(tiled[0], strip[0]), "forward differs"
    assert _rel(tiled[1], strip[1]) < 1e-5
    assert torch.equal(tiled[2], strip[2]), "data gradient differs"
    assert _rel(tiled[3], strip[3]) < 1e-5
    assert _rel(tiled[4], strip[4]) < 1e-5
