"""Numerics of every native gfx950 kernel against a plain PyTorch fp32 reference of the same op.

Inputs are rounded to bf16 first so the reference sees exactly the operands the kernel sees;
tolerances cover bf16 output rounding and fp32 accumulation-order differences.
"""
import pytest
import torch
import torch.nn.functional as TF

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel(a, b):
    a = a.float()
    b = b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def _cos(a, b):
    a = a.float().flatten()
    b = b.float().flatten()
    return (a @ b / (a.norm() * b.norm()).clamp_min(1e-12)).item()


def _nhwc(t):
    return t.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


@pytest.fixture(scope="module", autouse=True)
def _ext():
    from deep_vision_amd._ext import lib

    lib()
    torch.manual_seed(0)


CONV_CASES = [
    # N, C, H, W, K, R, stride, pad, groups
    (2, 64, 14, 14, 64, 1, 1, 0, 1),
    (2, 64, 14, 14, 128, 3, 1, 1, 1),
    (2, 256, 14, 14, 128, 1, 2, 0, 1),
    (2, 64, 15, 13, 64, 1, 2, 0, 1),     # 1x1 stride-2 scatter dgrad, odd map: zero-filling epilogue
    (2, 64, 14, 16, 32, 1, 3, 0, 1),     # 1x1 stride-3 scatter: 8 zero siblings per written pixel
    (2, 3, 32, 32, 64, 7, 2, 3, 1),      # stem, C padded 3 -> 8
    (2, 32, 17, 15, 48, 3, 2, 1, 1),     # stride-2 3x3: divisibility-gather dgrad
    (2, 64, 9, 9, 255, 1, 1, 0, 1),      # YOLO head: 255 outputs (padded channel stride)
    (2, 96, 13, 13, 256, 5, 1, 2, 1),    # 5x5, C % 64 != 0 (generic K decode)
    (2, 128, 8, 8, 128, 3, 1, 1, 2),     # grouped
    (3, 200, 7, 7, 520, 1, 1, 0, 1),     # odd M / N tails
    # strided dgrads by output parity (ops.conv._subpixel_dgrad): 3x3/2 (YOLOv3, ResNet-34),
    # odd maps, 4x4/2 (PatchGAN), 5x5/2 pad 2 (DCGAN), 3x3/3
    (2, 64, 17, 15, 64, 3, 2, 1, 1),
    (2, 128, 16, 16, 64, 3, 2, 1, 1),
    (2, 64, 16, 16, 128, 4, 2, 1, 1),
    (2, 64, 14, 14, 128, 5, 2, 2, 1),
    (2, 64, 13, 11, 64, 3, 3, 1, 1),
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_bwd(case):
    from deep_vision_amd import ops as F

    N, C, H, W, K, R, s, p, g = case
    x32 = torch.randn(N, C, H, W, device=DEV).bfloat16().float()
    w = (torch.randn(K, C // g, R, R, device=DEV) * (2.0 / (C * R * R / g)) ** 0.5).requires_grad_(True)
    x = _nhwc(x32).requires_grad_(True)
    y = F.conv2d(x, w, None, s, p, 1, g)
    xr = x32.clone().requires_grad_(True)
    wr = w.detach().bfloat16().float().requires_grad_(True)
    yr = TF.conv2d(xr, wr, None, s, p, 1, g)
    assert y.shape == yr.shape
    assert _rel(y, yr) < 2e-2
    dy32 = torch.randn_like(yr).bfloat16().float()
    y.backward(_nhwc(dy32))
    yr.backward(dy32)
    assert _rel(x.grad, xr.grad) < 3e-2
    assert _rel(w.grad, wr.grad) < 3e-2


def test_strided_dgrad_takes_subpixel_path():
    from deep_vision_amd import ops as F
    from deep_vision_amd.ops import conv as C

    x = _nhwc(torch.randn(2, 64, 17, 15, device=DEV)).requires_grad_(True)
    w = torch.randn(64, 64, 3, 3, device=DEV) * 0.05
    n0, t0 = C.COUNTERS_DGRAD["subpixel"], C.COUNTERS_DGRAD["tgather"]
    F.conv2d(x, w, None, 2, 1).sum().backward()
    assert C.COUNTERS_DGRAD["subpixel"] - n0 == 4 and C.COUNTERS_DGRAD["tgather"] == t0


@pytest.mark.parametrize("graph", [False, True])
def test_subpixel_parts_on_side_streams_match_one_stream(graph):
    """The parity parts launched side by side (ops.conv.SUBPIXEL_CONC) write disjoint pixels: the
    input gradient is bitwise the one-stream one, eager and inside a captured graph."""
    from deep_vision_amd.ops import conv as C

    dy = _nhwc(torch.randn(4, 128, 26, 26, device=DEV)).bfloat16()
    w = torch.randn(128, 64, 3, 3, device=DEV) * 0.05

    def run(conc):
        old, C.SUBPIXEL_CONC = C.SUBPIXEL_CONC, conc
        try:
            if not graph:
                return C._dgrad(dy, w, (4, 64, 52, 52), 64, 1, (2, 2), (1, 1), (1, 1), dy.device).clone()
            C._dgrad(dy, w, (4, 64, 52, 52), 64, 1, (2, 2), (1, 1), (1, 1), dy.device)  # warm the weight cache
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
                out = C._dgrad(dy, w, (4, 64, 52, 52), 64, 1, (2, 2), (1, 1), (1, 1), dy.device)
            g.replay()
            torch.cuda.synchronize()
            return out.clone()
        finally:
            C.SUBPIXEL_CONC = old

    a, b = run(False), run(True)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


def test_conv_bias_relu_epilogue():
    from deep_vision_amd import ops as F

    x32 = torch.randn(2, 32, 12, 12, device=DEV).bfloat16().float()
    w = torch.randn(40, 32, 3, 3, device=DEV) * 0.1
    b = torch.randn(40, device=DEV)
    y = F.conv2d(_nhwc(x32), w, b, 1, 1, act="relu")
    yr = TF.relu(TF.conv2d(x32, w.bfloat16().float(), b, 1, 1))
    assert _rel(y, yr) < 2e-2


def test_conv_stats_epilogue_and_bn():
    from deep_vision_amd import nn, ops as F

    torch.manual_seed(7)  # independent of the order / number of earlier cases in this module
    conv = nn.Conv2d(64, 128, 3, padding=1, bias=False).to(DEV)
    bn = nn.BatchNorm2d(128).to(DEV)
    bn.weight.data.uniform_(0.5, 1.5)
    bn.bias.data.uniform_(-0.5, 0.5)
    conv_r = torch.nn.Conv2d(64, 128, 3, padding=1, bias=False).to(DEV)
    bn_r = torch.nn.BatchNorm2d(128).to(DEV)
    conv_r.weight.data.copy_(conv.weight.data.bfloat16().float())
    bn_r.load_state_dict(bn.state_dict())
    x32 = torch.randn(4, 64, 16, 16, device=DEV).bfloat16().float()
    res32 = torch.randn(4, 128, 16, 16, device=DEV).bfloat16().float()
    x = _nhwc(x32).requires_grad_(True)
    res = _nhwc(res32).requires_grad_(True)
    y = F.conv_bn_act(x, conv, bn, "relu", residual=res)
    xr = x32.clone().requires_grad_(True)
    rr = res32.clone().requires_grad_(True)
    yr = TF.relu(bn_r(conv_r(xr)) + rr)
    assert _rel(y, yr) < 3e-2
    assert torch.allclose(bn.running_mean, bn_r.running_mean, atol=1e-2, rtol=1e-2)
    assert torch.allclose(bn.running_var, bn_r.running_var, atol=1e-2, rtol=2e-2)
    dy32 = torch.randn_like(yr).bfloat16().float()
    y.backward(_nhwc(dy32))
    yr.backward(dy32)
    # a ReLU-mask flip at z ~ 0 moves single elements by a whole gradient term: the max-based
    # bound is loose, the cosine is the tight one
    assert _rel(x.grad, xr.grad) < 0.15 and _cos(x.grad, xr.grad) > 0.999
    # ReLU-mask boundary elements (z ~ 0) can flip under bf16 rounding: compare globally
    assert _cos(res.grad, rr.grad) > 0.999
    mism = ((res.grad.float() - rr.grad).abs() > 0.05).float().mean().item()
    assert mism < 5e-3
    for a, b in ((bn.weight.grad, bn_r.weight.grad), (bn.bias.grad, bn_r.bias.grad),
                 (conv.weight.grad, conv_r.weight.grad)):
        assert _rel(a, b) < 8e-2 and _cos(a, b) > 0.999


def test_bn_eval():
    from deep_vision_amd import nn

    bn = nn.BatchNorm2d(48).to(DEV).eval()
    bn.running_mean.uniform_(-1, 1)
    bn.running_var.uniform_(0.5, 2)
    x32 = torch.randn(2, 48, 5, 5, device=DEV).bfloat16().float()
    y = bn(_nhwc(x32))
    yr = torch.nn.functional.batch_norm(x32, bn.running_mean, bn.running_var, bn.weight, bn.bias, False)
    assert _rel(y, yr) < 1e-2


@pytest.mark.parametrize("cfg", [(3, 2, 1, False), (3, 2, 0, True), (2, 2, 0, False), (3, 1, 1, False)])
def test_maxpool(cfg):
    from deep_vision_amd import ops as F

    k, s, p, ceil = cfg
    x32 = torch.randn(2, 64, 15, 15, device=DEV).bfloat16().float()
    x = _nhwc(x32).requires_grad_(True)
    xr = x32.clone().requires_grad_(True)
    y = F.max_pool2d(x, k, s, p, ceil)
    yr = TF.max_pool2d(xr, k, s, p, ceil_mode=ceil)
    assert y.shape == yr.shape
    assert _rel(y, yr) == 0.0
    dy = torch.randn_like(yr).bfloat16().float()
    y.backward(_nhwc(dy))
    yr.backward(dy)
    assert _rel(x.grad, xr.grad) < 1e-2


@pytest.mark.parametrize("cfg", [(7, 1, 0, False, True), (5, 3, 0, False, True), (3, 2, 1, True, False)])
def test_avgpool(cfg):
    from deep_vision_amd import ops as F

    k, s, p, ceil, cip = cfg
    x32 = torch.randn(2, 32, 14, 14, device=DEV).bfloat16().float()
    x = _nhwc(x32).requires_grad_(True)
    xr = x32.clone().requires_grad_(True)
    y = F.avg_pool2d(x, k, s, p, ceil, cip)
    yr = TF.avg_pool2d(xr, k, s, p, ceil, cip)
    assert y.shape == yr.shape
    assert _rel(y, yr) < 1e-2
    dy = torch.randn_like(yr).bfloat16().float()
    y.backward(_nhwc(dy))
    yr.backward(dy)
    assert _rel(x.grad, xr.grad) < 1e-2


def test_gap_linear_xent():
    from deep_vision_amd import ops as F

    x32 = torch.randn(8, 256, 7, 7, device=DEV).bfloat16().float()
    w = (torch.randn(100, 256, device=DEV) * 0.05).requires_grad_(True)
    b = torch.randn(100, device=DEV).requires_grad_(True)
    lab = torch.randint(0, 100, (8,), device=DEV)
    x = _nhwc(x32).requires_grad_(True)
    h = F.adaptive_avg_pool2d(x, 1).flatten(1)
    logits = F.linear(h, w, b)
    loss = F.cross_entropy(logits, lab)
    xr = x32.clone().requires_grad_(True)
    wr = w.detach().bfloat16().float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    hr = TF.adaptive_avg_pool2d(xr, 1).flatten(1).bfloat16().float()
    lr = TF.linear(hr, wr, br)
    lossr = TF.cross_entropy(lr, lab)
    assert abs(loss.item() - lossr.item()) < 2e-2 * max(1.0, abs(lossr.item()))
    loss.backward()
    lossr.backward()
    assert _rel(x.grad, xr.grad) < 5e-2
    assert _rel(w.grad, wr.grad) < 5e-2
    assert _rel(b.grad, br.grad) < 5e-2


def test_xent_retain_graph_twice():
    """a second backward through a retained graph gets the same (scaled) gradient."""
    from deep_vision_amd import ops as F

    logits = torch.randn(16, 100, device=DEV).requires_grad_(True)
    lab = torch.randint(0, 100, (16,), device=DEV)
    loss = F.cross_entropy(logits, lab)
    (loss * 3).backward(retain_graph=True)
    g1 = logits.grad.clone()
    logits.grad = None
    (loss * 3).backward()
    lr =logits.detach().clone().requires_grad_(True)
    (TF.cross_entropy(lr, lab) * 3).backward()
    assert _rel(g1, lr.grad) < 1e-3
    assert _rel(logits.grad, lr.grad) < 1e-3


def test_linear_odd_sizes():
    from deep_vision_amd import ops as F

    x32 = torch.randn(5, 100, device=DEV).bfloat16().float()
    w = (torch.randn(37, 100, device=DEV) * 0.1).requires_grad_(True)
    x = x32.clone().requires_grad_(True)
    y = F.linear(x, w, None, act="relu")
    wr = w.detach().bfloat16().float().requires_grad_(True)
    xr = x32.clone().requires_grad_(True)
    yr = TF.relu(TF.linear(xr, wr))
    assert _rel(y, yr) < 2e-2
    g = torch.randn_like(yr)
    y.backward(g)
    yr.backward(g.bfloat16().float())
    assert _rel(x.grad, xr.grad) < 5e-2
    assert _rel(w.grad, wr.grad) < 5e-2


@pytest.mark.parametrize("shape", [(128, 25088, 4096, True), (128, 4096, 4096, True), (64, 9216, 1000, False),
                                   (8, 2048, 1000, True)])
def test_linear_splitk(shape):
    """Short-M Linear layers (VGG16 fc6/fc7, AlexNet fc6 at batch 64, ResNet fc at batch 8) run
    with the K loop split over blocks and an ordered fp32 slab reduction (fwd and dgrad)."""
    from deep_vision_amd import ops as F
    from deep_vision_amd.ops.conv import gemm_ksplit

    N, K, O, bias = shape
    assert gemm_ksplit(N, O, K) > 1
    x32 = torch.randn(N, K, device=DEV).bfloat16().float()
    w = (torch.randn(O, K, device=DEV) * K ** -0.5).requires_grad_(True)
    b = torch.randn(O, device=DEV).requires_grad_(True) if bias else None
    x = x32.clone().to(torch.bfloat16).requires_grad_(True)
    y = F.linear(x, w, b, act="relu")
    wr = w.detach().bfloat16().float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True) if bias else None
    xr = x32.clone().requires_grad_(True)
    yr = TF.relu(TF.linear(xr, wr, br))
    assert _rel(y, yr) < 2e-2
    g = torch.randn_like(yr).bfloat16().float()
    y.backward(g.to(torch.bfloat16))
    yr.backward(g)
    assert _rel(x.grad, xr.grad) < 3e-2 and _cos(x.grad, xr.grad) > 0.9999
    assert _rel(w.grad, wr.grad) < 3e-2
    if bias:  # native column sum of the bf16 gradient rows
        assert _rel(b.grad, br.grad) < 1e-2
    if bias:
        assert _rel(b.grad, br.grad) < 2e-2
    y2 = F.linear(x.detach(), w.detach(), None if b is None else b.detach(), act="relu")
    assert torch.equal(F.linear(x.detach(), w.detach(), None if b is None else b.detach(), act="relu"), y2)


@pytest.mark.parametrize("case", [(32, 128, 8, 128, 3), (32, 256, 4, 256, 3), (8, 512, 7, 512, 1)])
def test_conv_splitk_small_maps(case):
    """Small output grids (Hourglass 4x4 / 8x8 scales) run split-K with the bias, residual and
    BatchNorm statistics applied by the finalize pass."""
    from deep_vision_amd import nn, ops as F
    from deep_vision_amd.ops.conv import conv_ksplit

    N, C, H, O, k = case
    assert conv_ksplit(N * H * H, O, k * k * C) > 1
    x32 = torch.randn(N, C, H, H, device=DEV).bfloat16().float()
    w = (torch.randn(O, C, k, k, device=DEV) * (2.0 / (C * k * k)) ** 0.5).requires_grad_(True)
    b = torch.randn(O, device=DEV).requires_grad_(True)
    r32 = torch.randn(N, O, H, H, device=DEV).bfloat16().float()
    x = _nhwc(x32).requires_grad_(True)
    res = _nhwc(r32).requires_grad_(True)
    y = F.conv2d(x, w, b, 1, k // 2, residual=res)
    xr, rr = x32.clone().requires_grad_(True), r32.clone().requires_grad_(True)
    wr = w.detach().bfloat16().float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    yr = TF.conv2d(xr, wr, br, 1, k // 2) + rr
    assert _rel(y, yr) < 2e-2
    g = torch.randn_like(yr).bfloat16().float()
    y.backward(_nhwc(g))
    yr.backward(g)
    assert _rel(x.grad, xr.grad) < 3e-2 and _rel(w.grad, wr.grad) < 3e-2
    assert _rel(b.grad, br.grad) < 1e-2 and _rel(res.grad, rr.grad) < 1e-2
    # conv -> BN -> ReLU with the statistics from the finalize pass
    conv = nn.Conv2d(C, O, k, padding=k // 2).to(DEV)
    bn = nn.BatchNorm2d(O).to(DEV)
    yb = F.conv_bn_act(_nhwc(x32), conv, bn, "relu")
    cr = torch.nn.Conv2d(C, O, k, padding=k // 2).to(DEV)
    cr.weight.data.copy_(conv.weight.data.bfloat16().float())
    cr.bias.data.copy_(conv.bias.data)
    ybr = TF.relu(TF.batch_norm(cr(x32), None, None, None, None, True, 0.1, bn.eps))
    assert _rel(yb, ybr) < 3e-2
    assert torch.allclose(bn.running_mean, 0.1 * cr(x32).mean((0, 2, 3)), atol=2e-3, rtol=2e-2)


def test_conv_transpose():
    from deep_vision_amd import ops as F

    for (cin, cout, k, s, p, op) in [(64, 32, 3, 2, 1, 1), (32, 16, 5, 1, 2, 0), (16, 8, 4, 2, 1, 0)]:
        x32 = torch.randn(2, cin, 7, 7, device=DEV).bfloat16().float()
        w = (torch.randn(cin, cout, k, k, device=DEV) * 0.1).requires_grad_(True)
        x = _nhwc(x32).requires_grad_(True)
        y = F.conv_transpose2d(x, w, None, s, p, op)
        xr = x32.clone().requires_grad_(True)
        wr = w.detach().bfloat16().float().requires_grad_(True)
        yr = TF.conv_transpose2d(xr, wr, None, s, p, op)
        assert y.shape == yr.shape, (y.shape, yr.shape)
        assert _rel(y, yr) < 2e-2
        dy = torch.randn_like(yr).bfloat16().float()
        y.backward(_nhwc(dy))
        yr.backward(dy)
        assert _rel(x.grad, xr.grad) < 3e-2
        assert _rel(w.grad, wr.grad) < 3e-2


def test_activations_add_upsample():
    from deep_vision_amd import ops as F

    x32 = torch.randn(2, 16, 6, 6, device=DEV).bfloat16().float()
    for act, ref in [("relu", TF.relu), ("tanh", torch.tanh), ("sigmoid", torch.sigmoid),
                     ("leaky", lambda t: TF.leaky_relu(t, 0.1))]:
        x = _nhwc(x32).requires_grad_(True)
        y = F.activation(x, act, 0.1)
        xr = x32.clone().requires_grad_(True)
        yr = ref(xr)
        assert _rel(y, yr) < 1e-2
        y.sum().backward()
        yr.sum().backward()
        assert _rel(x.grad, xr.grad) < 2e-2
    a = _nhwc(x32)
    y = F.add(a, a, act="relu")
    assert _rel(y, TF.relu(2 * x32)) < 1e-2
    x = _nhwc(x32).requires_grad_(True)
    u = F.upsample_nearest(x, 2)
    ur = TF.interpolate(x32, scale_factor=2, mode="nearest")
    assert _rel(u, ur) == 0.0
    u.sum().backward()
    assert torch.allclose(x.grad.float(), torch.full_like(x32, 4.0))


def test_upsample_add_matches_reference():
    """The fused Hourglass level merge: upsample_nearest(low) + skip, both gradients."""
    from deep_vision_amd import ops as F

    low32 = torch.randn(3, 64, 4, 4, device=DEV).bfloat16().float()
    skip32 = torch.randn(3, 64, 8, 8, device=DEV).bfloat16().float()
    low = _nhwc(low32).requires_grad_(True)
    skip = _nhwc(skip32).requires_grad_(True)
    y = F.upsample_add(low, skip, 2)
    lr_ = low32.clone().requires_grad_(True)
    sr = skip32.clone().requires_grad_(True)
    yr = TF.interpolate(lr_, scale_factor=2, mode="nearest") + sr
    assert _rel(y, yr) < 1e-2
    dy = torch.randn_like(yr).bfloat16().float()
    y.backward(_nhwc(dy))
    yr.backward(dy)
    assert _rel(low.grad, lr_.grad) < 1e-2
    assert _rel(skip.grad, sr.grad) == 0.0


def test_dropout_mask_consistency():
    from deep_vision_amd import ops as F

    x = torch.ones(4096, device=DEV, dtype=torch.bfloat16).requires_grad_(True)
    y = F.dropout(x, 0.5, True)
    kept = (y != 0).float().mean().item()
    assert 0.45 < kept < 0.55
    y.sum().backward()
    assert torch.equal((x.grad != 0), (y != 0))


def test_optimizers_match_torch():
    from deep_vision_amd.train.optim import FusedAdam, FusedRMSprop, FusedSGD

    for cls, ref_cls, kw in [
        (FusedSGD, torch.optim.SGD, dict(lr=0.1, momentum=0.9, weight_decay=1e-4)),
        (FusedAdam, torch.optim.Adam, dict(lr=1e-3)),
        (FusedRMSprop, torch.optim.RMSprop, dict(lr=0.045, alpha=0.9, eps=1.0)),
    ]:
        p1 = [torch.randn(33, 7, device=DEV, requires_grad=True), torch.randn(5, device=DEV, requires_grad=True)]
        p2 = [p.detach().clone().requires_grad_(True) for p in p1]
        o1 = cls(p1, **kw)
        o2 = ref_cls(p2, **kw)
        for _ in range(3):
            for a, b in zip(p1, p2):
                g = torch.randn_like(a)
                a.grad = g.clone()
                b.grad = g.clone()
            o1.step()
            o2.step()
        for a, b in zip(o1.param_views(), p2):
            assert torch.allclose(a, b, atol=1e-5, rtol=1e-4), cls.__name__


@pytest.mark.parametrize("cfg", [(32, 3, 1, 1), (64, 3, 2, 1), (128, 3, 1, 1), (1024, 3, 1, 1), (48, 5, 2, 2),
                                 (1040, 3, 2, 1), (64, 3, 2, 0), (16, 3, 1, 1), (24, 7, 1, 3), (40, 1, 2, 0)])
def test_depthwise(cfg):
    from deep_vision_amd import ops as F

    C, k, s, p = cfg
    x32 = torch.randn(2, C, 15, 13, device=DEV).bfloat16().float()
    w = (torch.randn(C, 1, k, k, device=DEV) * 0.3).requires_grad_(True)
    x = _nhwc(x32).requires_grad_(True)
    y = F.conv2d(x, w, None, s, p, 1, C)
    xr = x32.clone().requires_grad_(True)
    wr = w.detach().clone().requires_grad_(True)
    yr = TF.conv2d(xr, wr, None, s, p, 1, C)
    assert y.shape == yr.shape
    assert _rel(y, yr) < 2e-2
    dy = torch.randn_like(yr).bfloat16().float()
    y.backward(_nhwc(dy))
    yr.backward(dy)
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(w.grad, wr.grad) < 2e-2


def test_depthwise_bn_stats_fusion():
    from deep_vision_amd import nn, ops as F

    conv = nn.Conv2d(64, 64, 3, padding=1, groups=64, bias=False).to(DEV)
    bn = nn.BatchNorm2d(64).to(DEV)
    x32 = torch.randn(4, 64, 14, 14, device=DEV).bfloat16().float()
    y = F.conv_bn_act(_nhwc(x32), conv, bn, "relu")
    bn_r = torch.nn.BatchNorm2d(64).to(DEV)
    yr = TF.relu(bn_r(TF.conv2d(x32, conv.weight.detach(), None, 1, 1, 1, 64)))
    assert _rel(y, yr) < 3e-2


@pytest.mark.parametrize("mode", ["torch", "tf"])
def test_lrn(mode):
    from deep_vision_amd.ops import lrn

    for C, size in [(96, 96), (64, 5), (192, 192)]:
        x32 = torch.randn(2, C, 6, 5, device=DEV).bfloat16().float()
        x = _nhwc(x32).requires_grad_(True)
        xr = x32.clone().requires_grad_(True)
        if mode == "torch":
            y = lrn.local_response_norm(x, size, 1e-4, 0.75, 1.0)
            yr = TF.local_response_norm(xr, size, 1e-4, 0.75, 1.0)
        else:
            y = lrn.tf_local_response_norm(x, 5, 1.0, 1.0, 0.5)
            yr = lrn.tf_local_response_norm(xr, 5, 1.0, 1.0, 0.5)
        assert _rel(y, yr) < 2e-2
        dy = torch.randn_like(yr).bfloat16().float()
        y.backward(_nhwc(dy))
        yr.backward(dy)
        assert _rel(x.grad, xr.grad) < 3e-2


def test_grouped_padded_conv():
    from deep_vision_amd import ops as F

    for (C, O, G) in [(240, 60, 3), (60, 240, 3), (24, 48, 2)]:
        x32 = torch.randn(2, C, 9, 9, device=DEV).bfloat16().float()
        w = (torch.randn(O, C // G, 1, 1, device=DEV) * 0.1).requires_grad_(True)
        x = _nhwc(x32).requires_grad_(True)
        y = F.conv2d(x, w, None, 1, 0, 1, G)
        xr = x32.clone().requires_grad_(True)
        wr = w.detach().bfloat16().float().requires_grad_(True)
        yr = TF.conv2d(xr, wr, None, 1, 0, 1, G)
        assert y.shape == yr.shape
        assert _rel(y, yr) < 2e-2
        dy = torch.randn_like(yr).bfloat16().float()
        y.backward(_nhwc(dy))
        yr.backward(dy)
        assert _rel(x.grad, xr.grad) < 3e-2
        assert _rel(w.grad, wr.grad) < 3e-2


def test_conv_act_grad_from_concat_slice():
    """A fused conv+ReLU whose output feeds a channel concat receives a channel-slice gradient
    (pixel stride = concat width) -- Inception / YOLO routes."""
    from deep_vision_amd import ops as F

    x32 = torch.randn(2, 32, 9, 9, device=DEV).bfloat16().float()
    w1 = (torch.randn(24, 32, 1, 1, device=DEV) * 0.2).requires_grad_(True)
    w2 = (torch.randn(40, 32, 3, 3, device=DEV) * 0.1).requires_grad_(True)
    x = _nhwc(x32).requires_grad_(True)
    y = torch.cat([F.conv2d(x, w1, act="relu"), F.conv2d(x, w2, padding=1, act="relu")], 1)
    g = torch.randn(2, 64, 9, 9, device=DEV).bfloat16().float()  # the operands the kernels see
    y.backward(_nhwc(g))
    xr = x32.clone().requires_grad_(True)
    w1r = w1.detach().bfloat16().float().requires_grad_(True)
    w2r = w2.detach().bfloat16().float().requires_grad_(True)
    yr = torch.cat([TF.relu(TF.conv2d(xr, w1r)), TF.relu(TF.conv2d(xr, w2r, padding=1))], 1)
    yr.backward(g)
    assert _cos(x.grad, xr.grad) > 0.999
    assert _cos(w1.grad, w1r.grad) > 0.999 and _cos(w2.grad, w2r.grad) > 0.999


def test_batched_weight_prep_matches_per_layer():
    """ops.wcache: one batched launch after the optimizer step == the per-layer wprep kernel."""
    from deep_vision_amd.ops import wcache
    from deep_vision_amd.ops.common import ptr, stream_handle
    from deep_vision_amd.ops.conv import _prep_weight
    from deep_vision_amd._ext import lib

    wcache.clear()
    cases = [((64, 32, 3, 3), 1, 32, 0), ((64, 32, 3, 3), 1, 64, 1), ((48, 24, 1, 1), 2, 24, 0),
             ((48, 24, 1, 1), 2, 24, 1), ((100, 3, 7, 7), 1, 8, 0), ((100, 3, 7, 7), 1, 104, 1),
             ((1000, 2048, 1, 1), 1, 2048, 0), ((1000, 2048, 1, 1), 1, 1000, 1),
             ((96, 100, 3, 3), 1, 104, 0), ((64, 16, 3, 3), 4, 16, 0), ((32, 8, 5, 5), 1, 8, 0)]
    params = []
    for shape, G, pad, mode in cases:
        p = torch.nn.Parameter(torch.randn(*shape, device=DEV))
        _prep_weight(p, G, pad, mode)  # registers the cache entry
        params.append((p, G, pad, mode))
    with torch.no_grad():
        for p, *_ in params:
            p.mul_(-1.5)  # version bump: the batched refresh must rewrite everything
    wcache.after_step()
    for p, G, pad, mode in params:
        O, Ig, R, S = p.shape
        ref = torch.empty(G * (O // G if mode == 0 else Ig) * R * S * pad, dtype=torch.bfloat16, device=DEV)
        lib().wprep(ptr(p.detach()), ptr(ref), G, O // G, Ig, R, S, pad, mode, 0, stream_handle())
        got = _prep_weight(p, G, pad, mode)  # cache hit
        assert torch.equal(got, ref), (p.shape, G, pad, mode)
    # mode 2: the tap-packed stem layout (filter width padded to Sp, 4 channels)
    from deep_vision_amd.ops.conv import _prep_stem_weight

    stems = [(torch.nn.Parameter(torch.randn(64, 3, 7, 7, device=DEV)), 8),
             (torch.nn.Parameter(torch.randn(96, 3, 11, 11, device=DEV)), 16)]
    for p, Sp in stems:
        _prep_stem_weight(p, Sp)
        with torch.no_grad():
            p.mul_(0.5)
    wcache.after_step()
    for p, Sp in stems:
        O, I, R, S = p.shape
        ref = torch.empty(O * R * Sp * 4, dtype=torch.bfloat16, device=DEV)
        lib().wprep(ptr(p.detach()), ptr(ref), 1, O, I, R, S, 4, 2, Sp, stream_handle())
        assert torch.equal(_prep_stem_weight(p, Sp), ref), (p.shape, Sp)
    wcache.clear()


STEM_CASES = [
    # N, C, H, W, K, R, S, stride, padding (int | (top, bottom, left, right)), bias, act
    (2, 3, 32, 32, 64, 7, 7, 2, 3, False, None),         # ResNet / Inception stem
    (2, 3, 36, 36, 96, 11, 11, 4, 2, True, "relu"),      # AlexNet V1 conv1 (Sp = 16)
    (2, 3, 30, 30, 32, 5, 5, 2, 2, True, None),          # 5x5 s2
    (3, 3, 32, 32, 128, 7, 7, 2, (2, 3, 2, 3), False, None),  # Keras 'same' 7x7 s2 (Hourglass stem)
    (2, 1, 28, 28, 40, 5, 5, 2, 2, False, "relu"),       # 1 input channel
]


@pytest.mark.parametrize("case", STEM_CASES)
def test_stem_packed_conv(case):
    """Tap-packed stem path (ops.conv._StemConvFn, csrc conv_fwd packed mode + wgrad ldx=4) vs torch."""
    from deep_vision_amd import ops as F
    from deep_vision_amd.ops import conv as C

    N, Cin, H, W, K, R, S, s, p, has_b, act = case
    x = torch.randn(N, Cin, H, W, device=DEV).bfloat16().float()
    w = (torch.randn(K, Cin, R, S, device=DEV) * 0.1).requires_grad_(True)
    b = torch.randn(K, device=DEV).requires_grad_(True) if has_b else None
    pad, extra = C.norm_padding(p)
    assert C._stem_geometry(x, w, (s, s), pad, (1, 1), 1, extra) is not None
    y = F.conv2d(x, w, b, s, p, act=act)
    wr = w.detach().bfloat16().float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True) if has_b else None
    xr = TF.pad(x, (p[2], p[3], p[0], p[1])) if isinstance(p, tuple) else x
    yr = TF.conv2d(xr, wr, br, s, 0 if isinstance(p, tuple) else p)
    if act == "relu":
        yr = TF.relu(yr)
    assert y.shape == yr.shape
    assert _rel(y, yr) < 2e-2
    dy = torch.randn_like(yr).bfloat16().float()
    y.backward(_nhwc(dy))
    yr.backward(dy)
    assert _rel(w.grad, wr.grad) < 3e-2
    if has_b:
        assert _rel(b.grad, br.grad) < 3e-2


STEM_KERNEL_CASES = [
    # N, C, H, W, padding, bias, act
    (3, 3, 64, 64, 3, False, None),            # ResNet / Inception stem geometry (Q = 32)
    (2, 3, 50, 38, 3, True, "relu"),           # Q = 19: partial 16-pixel fragments, ragged row groups
    (2, 3, 45, 61, (2, 3, 2, 3), False, "leaky"),  # Keras 'same' 7x7 s2 (Hourglass), odd sizes
    (5, 1, 30, 30, 3, True, None),             # one input channel, 5 images (several blocks per image)
    (8, 3, 96, 96, 3, False, None),            # P = 48 over 8 images: rows per block do not divide P evenly
]


@pytest.mark.parametrize("case", STEM_KERNEL_CASES)
def test_stem_dedicated_kernel(case):
    """csrc/stem.hip (7x7, 64 output channels) forward, BN statistics and weight gradient (into a
    zero and into a live gradient buffer) vs the fp32 torch conv of the same bf16 operands."""
    from deep_vision_amd import ops as F
    from deep_vision_amd.ops import conv as C

    N, Cin, H, W, p, has_b, act = case
    torch.manual_seed(1)
    x = torch.randn(N, Cin, H, W, device=DEV).bfloat16().float()
    w = (torch.randn(64, Cin, 7, 7, device=DEV) * 0.1).requires_grad_(True)
    b = torch.randn(64, device=DEV).requires_grad_(True) if has_b else None
    n0 = dict(C.COUNTERS)
    y = F.conv2d(x, w, b, 2, p, act=act, slope=0.1)
    assert C.COUNTERS["stem_kernel_fwd"] == n0["stem_kernel_fwd"] + 1, "dedicated stem kernel not taken"
    wr = w.detach().bfloat16().float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True) if has_b else None
    xr = TF.pad(x, (p[2], p[3], p[0], p[1])) if isinstance(p, tuple) else x
    yr = TF.conv2d(xr, wr, br, 2, 0 if isinstance(p, tuple) else p)
    if act == "relu":
        yr = TF.relu(yr)
    elif act == "leaky":
        yr = TF.leaky_relu(yr, 0.1)
    assert y.shape == yr.shape
    assert _rel(y, yr) < 1e-2
    dy = torch.randn_like(yr).bfloat16().float()
    y.backward(_nhwc(dy))
    yr.backward(dy)
    assert C.COUNTERS["stem_kernel_wgrad"] == n0["stem_kernel_wgrad"] + 1
    assert _rel(w.grad, wr.grad) < 1e-2
    # second backward accumulates into the live gradient
    y2 = F.conv2d(x, w, b, 2, p, act=act, slope=0.1)
    y2.backward(_nhwc(dy))
    assert _rel(w.grad, 2 * wr.grad) < 1e-2
    if has_b:
        assert _rel(b.grad, 2 * br.grad) < 2e-2


def test_stem_dedicated_kernel_stats():
    """Stem BN statistics from the dedicated kernel's register accumulators (shifted sums)."""
    from deep_vision_amd import nn
    from deep_vision_amd import ops as F
    from deep_vision_amd.ops import conv as C

    conv = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).to(DEV)
    bn = nn.BatchNorm2d(64).to(DEV)
    ref_conv = torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).to(DEV)
    ref_conv.weight.data.copy_(conv.weight.data.bfloat16().float())
    ref_bn = torch.nn.BatchNorm2d(64).to(DEV)
    n0 = C.COUNTERS["stem_kernel_fwd"]
    for it in range(3):  # shifted sums: the shift is the previous batch's mean from step 2 on
        x = (torch.randn(3, 3, 72, 60, device=DEV) * 2 + 5).bfloat16().float()
        y = F.conv_bn_act(x, conv, bn, "relu")
        yr = TF.relu(ref_bn(ref_conv(x)))
        assert _rel(y, yr) < 3e-2, it
    assert C.COUNTERS["stem_kernel_fwd"] == n0 + 3
    assert _rel(bn.running_mean, ref_bn.running_mean) < 1e-2
    assert _rel(bn.running_var, ref_bn.running_var) < 1e-2


def test_stem_conv_bn_stats():
    """Stem conv with BatchNorm statistics from the packed kernel's epilogue (ResNet stem)."""
    from deep_vision_amd import nn
    from deep_vision_amd import ops as F

    conv = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).to(DEV)
    bn = nn.BatchNorm2d(64).to(DEV)
    x = torch.randn(4, 3, 64, 64, device=DEV).bfloat16().float()
    y = F.conv_bn_act(x, conv, bn, "relu")
    ref_conv = torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).to(DEV)
    ref_conv.weight.data.copy_(conv.weight.data.bfloat16().float())
    ref_bn = torch.nn.BatchNorm2d(64).to(DEV)
    yr = TF.relu(ref_bn(ref_conv(x)))
    assert _rel(y, yr) < 3e-2
    assert _rel(bn.running_mean, ref_bn.running_mean) < 2e-2
    assert _rel(bn.running_var, ref_bn.running_var) < 2e-2


def test_deterministic_wgrad_bitwise():
    """set_deterministic(): split-K weight gradients are bitwise reproducible (slab reduction in a
    fixed order), and equal to the atomic path up to fp32 summation order."""
    import deep_vision_amd as dv
    from deep_vision_amd import ops as F

    x = _nhwc(torch.randn(16, 64, 28, 28, device=DEV)).requires_grad_(False)
    w = (torch.randn(128, 64, 3, 3, device=DEV) * 0.05).requires_grad_(True)
    dy = _nhwc(torch.randn(16, 128, 28, 28, device=DEV))
    grads = []
    try:
        dv.set_deterministic(True)
        for _ in range(3):
            w.grad = None
            F.conv2d(x, w, None, 1, 1).backward(dy)
            grads.append(w.grad.clone())
    finally:
        dv.set_deterministic(False)
    assert torch.equal(grads[0], grads[1]) and torch.equal(grads[1], grads[2])
    w.grad = None
    F.conv2d(x, w, None, 1, 1).backward(dy)
    assert _rel(w.grad, grads[0]) < 1e-5


def test_sync_check_mode_runs():
    import deep_vision_amd as dv
    from deep_vision_amd import ops as F
    from deep_vision_amd._ext import lib

    try:
        dv.set_sync_check(True)
        assert lib().sync_check()
        y = F.conv2d(_nhwc(torch.randn(2, 64, 8, 8, device=DEV)), torch.randn(64, 64, 3, 3, device=DEV), None, 1, 1)
        assert torch.isfinite(y).all()
    finally:
        dv.set_sync_check(False)


@pytest.mark.parametrize("case", [
    # N, C, H, W, K, R, pad, bias, input needs grad
    (2, 256, 16, 16, 256, 3, 1, False, True),   # CycleGAN ResNet block conv
    (2, 3, 32, 32, 64, 7, 3, False, False),     # generator stem on the network input (tap-packed)
    (2, 3, 32, 32, 64, 7, 3, False, True),      # stem on a generated image (cycle loss: needs dX)
    (2, 64, 20, 18, 3, 7, 3, True, True),       # output conv 64 -> 3 with bias
])
def test_reflect_pad_fused_conv(case):
    """ReflectionPad2d fused into the im2col gather (pad_mode='reflect'): forward, dgrad (padded-grid
    dgrad + border fold) and wgrad (mirrored taps) vs torch pad(reflect) + conv in fp32."""
    from deep_vision_amd import ops as F

    N, C, H, W, K, R, p, has_b, xg = case
    x32 = torch.randn(N, C, H, W, device=DEV).bfloat16().float()
    w = (torch.randn(K, C, R, R, device=DEV) * (2.0 / (C * R * R)) ** 0.5).requires_grad_(True)
    b = torch.randn(K, device=DEV).requires_grad_(True) if has_b else None
    x = (_nhwc(x32) if C % 8 == 0 else x32.clone()).requires_grad_(xg)
    y = F.conv2d(x, w, b, 1, p, pad_mode="reflect")
    xr = x32.clone().requires_grad_(xg)
    wr = w.detach().bfloat16().float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True) if has_b else None
    yr = TF.conv2d(TF.pad(xr, (p, p, p, p), mode="reflect"), wr, br)
    assert y.shape == yr.shape
    assert _rel(y, yr) < 2e-2
    dy32 = torch.randn_like(yr).bfloat16().float()
    y.backward(_nhwc(dy32) if K % 8 == 0 else dy32)
    yr.backward(dy32)
    assert _rel(w.grad, wr.grad) < 3e-2
    if xg:
        assert _rel(x.grad, xr.grad) < 3e-2
    if has_b:
        assert _rel(b.grad, br.grad) < 3e-2


@pytest.mark.parametrize("W", [224, 30])
def test_u8_normalize_kernel(W):
    """csrc u8_normalize: uint8 HWC crops + flip flags -> bf16 NCHW, vs the fp32 torch form."""
    from deep_vision_amd.data.device_input import normalize_u8

    x = torch.randint(0, 256, (5, 17, W, 3), dtype=torch.uint8)
    flip = torch.tensor([1, 0, 1, 1, 0], dtype=torch.bool)
    ref = normalize_u8(x, flip)
    out = normalize_u8(x.to(DEV), flip.to(DEV))
    assert out.dtype == torch.bfloat16 and tuple(out.shape) == (5, 3, 17, W)
    assert torch.allclose(out.float().cpu(), ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("H,W", [(224, 224), (320, 300), (9, 13)])
def test_u8_jitter_kernel_matches_worker_bytes(H, W):
    """csrc u8_jitter (ColorJitter on the GPU, in LDS for a 224x224 crop, in global memory above
    150 KB) gives exactly the bytes of the worker-side native jitter (PIL enhancer arithmetic) for
    every enhancer order, factors above / below 1 and a factor of exactly 1 (skipped)."""
    import itertools

    from deep_vision_amd.data.device_input import jitter_u8

    g = torch.Generator().manual_seed(H * W)
    orders = list(itertools.permutations(range(3)))
    N = len(orders) + 2
    x = torch.randint(0, 256, (N, H, W, 3), dtype=torch.uint8, generator=g)
    x[0] = 255 - x[0] // 3  # a bright image: clipping above
    f = 0.8 + 0.4 * torch.rand(N, 3, generator=g)
    f[1, 1] = 1.0
    o = torch.tensor(orders + [(0, 1, 2), (2, 0, 1)], dtype=torch.float32)
    prm = torch.cat([f, o], 1)
    ref = jitter_u8(x.clone(), prm)
    out = jitter_u8(x.to(DEV), prm.to(DEV)).cpu()
    assert not torch.equal(ref, x)
    assert torch.equal(out, ref)


@pytest.mark.parametrize("train", [True, False])
def test_conv_bias_grad_via_bn(train):
    """A conv bias feeding a training BatchNorm gets its gradient from the BN's backward sums
    (bn_bwd_finalize xsum, no reduction pass over dy): it must match the fp32 reference, where it is
    ~0 (the BN input gradient sums to zero per channel); eval statistics reduce dx explicitly."""
    from deep_vision_amd import nn, ops as F

    torch.manual_seed(5)
    conv = nn.Conv2d(64, 128, 1).to(DEV)
    bn = nn.BatchNorm2d(128).to(DEV)
    if not train:
        bn.eval()
        bn.running_mean.uniform_(-0.5, 0.5)
        bn.running_var.uniform_(0.5, 2.0)
    conv_r = torch.nn.Conv2d(64, 128, 1).to(DEV)
    bn_r = torch.nn.BatchNorm2d(128).to(DEV)
    conv_r.load_state_dict({k: v.bfloat16().float() if k == "weight" else v for k, v in conv.state_dict().items()})
    bn_r.load_state_dict(bn.state_dict())
    bn_r.train(train)
    x32 = torch.randn(4, 64, 12, 12, device=DEV).bfloat16().float()
    y = F.conv_bn_act(_nhwc(x32), conv, bn, "relu")
    yr = TF.relu(bn_r(conv_r(x32)))
    g = torch.randn_like(yr).bfloat16().float()
    y.backward(_nhwc(g))
    yr.backward(g)
    scale = conv_r.weight.grad.abs().max().item()
    assert conv.bias.grad is not None
    if train:
        assert (conv.bias.grad - conv_r.bias.grad).abs().max().item() < 1e-2 * scale
    else:
        assert _rel(conv.bias.grad, conv_r.bias.grad) < 3e-2


def test_darknet_residual_post_activation_add():
    """Darknet residual block: x + leaky(bn(conv3x3(leaky(bn(conv1x1(x)))))) with the add inside
    the BN apply pass (post-activation residual) and x's two gradients joined in conv_1x1's dgrad
    epilogue, against the same block on the PyTorch path (fp32)."""
    import copy

    from deep_vision_amd.models.yolov3 import DarknetResidual
    from deep_vision_amd.ops.common import set_backend

    torch.manual_seed(0)
    blk = DarknetResidual(32, 64).to(DEV)
    ref = copy.deepcopy(blk)
    x32 = torch.randn(4, 64, 20, 20, device=DEV).bfloat16().float()
    x = _nhwc(x32).requires_grad_(True)
    y = blk(x)
    dy = torch.randn(4, 64, 20, 20, device=DEV).bfloat16().float()
    y.backward(_nhwc(dy))
    set_backend("torch")
    try:
        xr = x32.clone().requires_grad_(True)
        yr = ref(xr)
        yr.backward(dy)
    finally:
        set_backend("native")
    assert _rel(y, yr) < 3e-2
    # leaky-ReLU slope flips at z ~ 0 under bf16 rounding move single elements: compare globally
    assert _cos(x.grad, xr.grad) > 0.999
    for (n, p), (_, q) in zip(blk.named_parameters(), ref.named_parameters()):
        assert _cos(p.grad, q.grad) > 0.998, n


@pytest.mark.parametrize("C,O,H,bnfuse", [(512, 1024, 13, False), (1024, 512, 13, True), (256, 256, 9, False)])
def test_dgrad_split_k_small_grid(C, O, H, bnfuse):
    """Stride-1 3x3 dgrads on under-filled grids split K across blocks (ops.conv.dgrad_ksplit:
    YOLOv3's 13x13 layers): against fp32 torch, with and without a BatchNorm in front (its
    backward sums then come from the split-K finalize pass that stores dX)."""
    from deep_vision_amd import nn, ops as F
    from deep_vision_amd.ops import conv as Cv

    torch.manual_seed(C + O)
    N = 2
    assert Cv.dgrad_ksplit(N * H * H, C, 9 * O) > 1
    x = torch.randn(N, C, H, H, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    conv = nn.Conv2d(C, O, 3, padding=1, bias=False).to(DEV)
    dy = torch.randn(N, O, H, H, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xi = x.clone().requires_grad_(True)
    if bnfuse:
        from deep_vision_amd.ops.bn import COUNTERS

        bn = nn.BatchNorm2d(C).to(DEV)
        h = F.batch_norm_act(xi, bn, "relu")
        y = F.conv2d(h, conv.weight, None, 1, 1)
        n0 = COUNTERS["bwd_reduce_fused"]
        y.backward(dy)
        # the BN-backward sums come from the split-K finalize pass (csrc/conv_fwd.hip FinBnr)
        assert COUNTERS["bwd_reduce_fused"] - n0 == (1 if Cv.FIN_BNR else 0)
        xr = x.float().requires_grad_(True)
        hr = torch.relu(torch.nn.functional.batch_norm(xr, None, None, bn.weight.float(), bn.bias.float(), True))
        yr = torch.nn.functional.conv2d(hr.to(torch.bfloat16).float(), conv.weight.to(torch.bfloat16).float(), None, 1, 1)
    else:
        y = F.conv2d(xi, conv.weight, None, 1, 1)
        y.backward(dy)
        xr = x.float().requires_grad_(True)
        yr = torch.nn.functional.conv2d(xr, conv.weight.to(torch.bfloat16).float(), None, 1, 1)
    yr.backward(dy.float())
    err = ((xi.grad.float() - xr.grad).norm() / xr.grad.norm()).item()
    assert err < 2e-2, err
