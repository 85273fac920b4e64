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
    assert stats.shape[0] == 129 and not stats[128].any()
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
