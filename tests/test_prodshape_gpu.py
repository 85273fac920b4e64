"""Numerics of the hot-path kernels at the shapes the ResNet-50 / MobileNet steps dispatch, against
an fp32 PyTorch reference of the same computation.

The unit tests in test_ops_gpu.py use toy maps (7-32 px, batch 2). Here every case runs at a
production shape so the kernels actually selected by the tile heuristics are the ones checked:
  * whole bottleneck blocks (conv -> BN -> ReLU x3, projection / identity shortcut, fused
    residual + ReLU, the BN-backward statistics folded into the dgrad epilogue, the gradient join
    of the shortcut) at stage-1/2/3 shapes, forward and every parameter gradient;
  * the 256x256 / 128-row-wave-tile forward variant (forced at a small batch);
  * split-K weight gradient with a reduction dimension of 200,704 pixels;
  * depthwise fwd/dgrad/wgrad at 112x112;
  * the tap-packed stem at 224x224.
The reference is the same module run through the torch backend in fp32 on bf16-rounded inputs; the forward is held to a few percent max error, every gradient to twice the deviation of
PyTorch's own bf16 (autocast) path from that fp32 reference (bf16 activations flip ReLU masks at
z ~ 0, which bounds the attainable gradient cosine at ~0.998 for a bottleneck block).
"""
import copy

import pytest
import torch
import torch.nn.functional as TF

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def _cos(a, b):
    a, b = a.float().flatten(), b.float().flatten()
    return (a @ b / (a.norm() * b.norm()).clamp_min(1e-12)).item()


def _nhwc(t):
    return t.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


@pytest.fixture(scope="module", autouse=True)
def _ext():
    from deep_vision_amd._ext import lib

    lib()
    torch.manual_seed(0)
    yield
    lib().conv_fwd_variant(0)


def _reference(module, x32, dy32, xgrad=True, autocast=False):
    """torch-backend forward/backward of a copy of ``module``: fp32, or PyTorch's own bf16 path
    (autocast) -- the precision-matched yardstick. Parameters are NOT rounded: the native path
    keeps BatchNorm affine and depthwise filters in fp32 and rounds only MFMA conv operands, as
    autocast does (rounding BN's beta in the reference alone shifts z and flips ReLU masks)."""
    from deep_vision_amd import ops as F

    ref = copy.deepcopy(module).float()
    xr = x32.clone().requires_grad_(xgrad)
    F.set_backend("torch")
    try:
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
            yr = ref(xr)
        yr.float().backward(dy32)
    finally:
        F.set_backend("native")
    return ref, xr, yr


def _check_module(module, x32, fwd_tol=3e-2, xgrad=True):
    """Native forward/backward vs fp32. A bf16 chain flips ReLU masks (and max-pool arg-maxes)
    wherever the fp32 pre-activation is within bf16 rounding of zero, so gradients are held to
    PyTorch's own bf16 path: 1 - cos(native, fp32) <= 2 * (1 - cos(autocast bf16, fp32)) + 2e-4."""
    x = _nhwc(x32).requires_grad_(xgrad)
    y = module(x)
    dy32 = torch.randn(y.shape, device=DEV).bfloat16().float()
    ref, xr, yr = _reference(module, x32, dy32, xgrad)
    ab, xb, _ = _reference(module, x32, dy32, xgrad, autocast=True)
    y.backward(_nhwc(dy32))
    assert y.shape == yr.shape
    assert _rel(y, yr) < fwd_tol, _rel(y, yr)

    def close(name, g, gr, gb):
        dn, db = 1 - _cos(g, gr), 1 - _cos(gb, gr)
        assert dn <= 2 * db + 2e-4, (name, dn, db)

    if xgrad:
        close("x", x.grad, xr.grad, xb.grad)
    for (name, p), pr, pb in zip(module.named_parameters(), ref.parameters(), ab.parameters()):
        assert p.grad is not None, name
        close(name, p.grad, pr.grad, pb.grad)
    return y


# (in, mid, out, stride, downsample, H, batch): ResNet-50 blocks at their stage shapes
BLOCKS = [
    (64, 64, 256, 1, True, 56, 32),      # conv2_x block 0: projection, 64-channel 3x3 at 56x56
    (256, 64, 256, 1, False, 56, 32),    # conv2_x identity block
    (256, 128, 512, 2, True, 56, 32),    # conv3_x block 0: stride on the first 1x1 (V1)
    (1024, 256, 1024, 1, False, 14, 64), # conv4_x identity block
    (2048, 512, 2048, 1, False, 7, 64),  # conv5_x identity block
]


@pytest.mark.parametrize("cfg", BLOCKS, ids=lambda c: f"{c[0]}-{c[1]}-{c[2]}s{c[3]}@{c[5]}b{c[6]}")
def test_bottleneck_block(cfg):
    from deep_vision_amd.models.resnet import BottleneckBlock, _init

    cin, mid, cout, s, ds, H, N = cfg
    torch.manual_seed(1)
    blk = BottleneckBlock(cin, mid, cout, stride=s, downsample=ds).to(DEV)
    _init(blk)
    for m in blk.modules():  # non-trivial BN affine parameters
        if isinstance(m, torch.nn.BatchNorm2d):
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.3, 0.3)
    x32 = torch.randn(N, cin, H, H, device=DEV).bfloat16().float()
    _check_module(blk, x32)


def test_bottleneck_block_big_tiles():
    """conv4_x identity block with the 256x256 tile / 128-row wave-tile forward forced on every
    eligible conv (N % 256 == 0, K >= 1024: conv1's dgrad, conv3, conv2's 3x3 at 256 channels)."""
    from deep_vision_amd._ext import lib
    from deep_vision_amd.models.resnet import BottleneckBlock, _init

    torch.manual_seed(2)
    blk = BottleneckBlock(1024, 256, 1024).to(DEV)
    _init(blk)
    x32 = torch.randn(16, 1024, 14, 14, device=DEV).bfloat16().float()
    lib().conv_fwd_variant(100)
    try:
        _check_module(blk, x32)
    finally:
        lib().conv_fwd_variant(0)


def test_conv_fwd_big_tile_epilogues():
    """256x256 / 128-row wave tiles with the bias+ReLU and residual-accumulate epilogues and an
    M tail (M = 2 * 13 * 13 = 338: the second 64-row pass of a wave is partly out of range)."""
    from deep_vision_amd._ext import lib
    from deep_vision_amd import ops as F

    x32 = torch.randn(2, 256, 13, 13, device=DEV).bfloat16().float()
    w = torch.randn(512, 256, 3, 3, device=DEV) * 0.03
    b = torch.randn(512, device=DEV)
    lib().conv_fwd_variant(100)
    try:
        y = F.conv2d(_nhwc(x32), w, b, 1, 1, act="relu")
    finally:
        lib().conv_fwd_variant(0)
    yr = TF.relu(TF.conv2d(x32, w.bfloat16().float(), b, 1, 1))
    assert _rel(y, yr) < 2e-2


def test_wgrad_splitk_200k():
    """3x3 64->64 at 56x56, batch 64: the weight-gradient reduction runs over 200,704 pixels."""
    from deep_vision_amd import ops as F

    x32 = torch.randn(64, 64, 56, 56, device=DEV).bfloat16().float()
    w = (torch.randn(64, 64, 3, 3, device=DEV) * 0.06).requires_grad_(True)
    y = F.conv2d(_nhwc(x32), w, None, 1, 1)
    dy32 = torch.randn(y.shape, device=DEV).bfloat16().float()
    y.backward(_nhwc(dy32))
    wr = w.detach().bfloat16().float().requires_grad_(True)
    TF.conv2d(x32, wr, None, 1, 1).backward(dy32)
    assert _rel(w.grad, wr.grad) < 1e-2
    assert _cos(w.grad, wr.grad) > 0.9999


@pytest.mark.parametrize("cfg", [(32, 112, 1), (64, 112, 2), (512, 14, 1)], ids=lambda c: f"c{c[0]}@{c[1]}s{c[2]}")
def test_depthwise_bn_relu_production(cfg):
    """MobileNet's depthwise -> BN -> ReLU at batch 64 (stats, mask bits and all three gradients)."""
    from deep_vision_amd import nn

    C, H, s = cfg

    class DwBlock(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.dw = nn.Conv2d(C, C, 3, stride=s, padding=1, groups=C, bias=False)
            self.bn = nn.BatchNorm2d(C)
            self.act = nn.ReLU(inplace=True)

        def forward(self, x):
            from deep_vision_amd import ops as F

            return F.conv_bn_act(x, self.dw, self.bn, "relu")

    torch.manual_seed(3)
    m = DwBlock().to(DEV)
    m.bn.weight.data.uniform_(0.5, 1.5)
    m.bn.bias.data.uniform_(-0.3, 0.3)
    x32 = torch.randn(64, C, H, H, device=DEV).bfloat16().float()
    _check_module(m, x32)


def test_stem_production():
    """ResNet-50 stem (7x7/2 conv -> BN -> ReLU -> 3x3/2 max-pool) at 224x224, batch 32."""
    from deep_vision_amd import nn

    class Stem(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
            self.bn1 = nn.BatchNorm2d(64)
            self.pool = nn.MaxPool2d(3, 2, 1)

        def forward(self, x):
            from deep_vision_amd import ops as F

            return self.pool(F.conv_bn_act(x, self.conv1, self.bn1, "relu"))

    torch.manual_seed(4)
    m = Stem().to(DEV)
    x32 = torch.randn(32, 3, 224, 224, device=DEV).bfloat16().float()
    _check_module(m, x32, xgrad=False)  # an image input needs no gradient: the tap-packed path


def _same_up_to_stat_rounding(a, b):
    """Equal except where the batch statistics' last fp32 bit moved an element across a bf16
    rounding boundary: the statistics are reduced with float atomics, so two runs of the same
    BatchNorm may differ in their summation order (a handful of elements by one bf16 ulp)."""
    a, b = a.float(), b.float()
    d = (a - b).abs()
    assert (d <= b.abs() * 2.0 ** -7 + 1e-30).all(), d.max().item()
    assert (d > 0).float().mean().item() < 1e-3


class _FusedStem(torch.nn.Module):
    """ResNet stem through the fused BN -> ReLU -> max-pool op (ops.bn._BNActPoolFn)."""

    def __init__(self, fused=True):
        super().__init__()
        from deep_vision_amd import nn

        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.pool = nn.MaxPool2d(3, 2, 1)
        self.fused = fused

    def forward(self, x):
        from deep_vision_amd import ops as F

        if self.fused:
            return F.conv_bn_act_maxpool(x, self.conv1, self.bn1, "relu", self.pool)
        return self.pool(F.conv_bn_act(x, self.conv1, self.bn1, "relu"))


def test_stem_fused_production():
    """Fused stem (BN apply + ReLU + max-pool in one pass, gather-form backward) at 224x224,
    batch 32, against the fp32 reference."""
    torch.manual_seed(4)
    m = _FusedStem().to(DEV)
    m.bn1.weight.data.uniform_(0.5, 1.5)
    m.bn1.bias.data.uniform_(-0.2, 0.2)
    x32 = torch.randn(32, 3, 224, 224, device=DEV).bfloat16().float()
    _check_module(m, x32, xgrad=False)


def test_stem_fused_matches_unfused():
    """The fused op reproduces the unfused native chain: identical pooled output (the BN output's
    bf16 rounding is kept before the max), equal running statistics, and gradients equal up to
    the order of the BN-backward reductions."""
    torch.manual_seed(5)
    a = _FusedStem(fused=True).to(DEV)
    b = _FusedStem(fused=False).to(DEV)
    b.load_state_dict(a.state_dict())
    for m in (a, b):
        m.bn1.weight.data.uniform_(0.5, 1.5)
    b.bn1.weight.data.copy_(a.bn1.weight.data)
    x = _nhwc(torch.randn(16, 3, 224, 224, device=DEV))
    ya, yb = a(x), b(x)
    _same_up_to_stat_rounding(ya, yb)
    dy = _nhwc(torch.randn(ya.shape, device=DEV))
    ya.backward(dy)
    yb.backward(dy)
    torch.cuda.synchronize()
    assert torch.allclose(a.bn1.running_mean, b.bn1.running_mean, rtol=1e-5, atol=1e-6)
    assert torch.allclose(a.bn1.running_var, b.bn1.running_var, rtol=1e-5, atol=1e-6)
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        assert _rel(pa.grad, pb.grad) < 2e-3, (n, _rel(pa.grad, pb.grad))


@pytest.mark.parametrize("cfg", [(64, 3, 2, 1, False, 29, 31, "relu"), (64, 3, 2, 1, False, 30, 32, "relu"),
                                 (32, 3, 2, 1, False, 30, 32, "leaky"), (64, 3, 2, 1, False, 29, 31, "leaky"),
                                 (32, 2, 2, 0, False, 29, 31, "relu"), (128, 3, 1, 1, False, 29, 31, "relu"),
                                 (16, 3, 2, 0, True, 29, 31, "relu")],
                         ids=lambda c: f"c{c[0]}k{c[1]}s{c[2]}p{c[3]}{'ceil' if c[4] else ''}_{c[5]}x{c[6]}_{c[7]}")
def test_bn_act_maxpool_windows(cfg):
    """Fused BN -> act -> max-pool vs the unfused native chain: the compiled 3x3/s2 window (integer-
    key ReLU forward; even maps take the 2x2-input-block backward, odd maps the per-input gather),
    LeakyReLU (float-compare forward) and the runtime-window form (2x2/s2, 3x3/s1, ceil mode)."""
    from deep_vision_amd import nn
    from deep_vision_amd import ops as F

    C, k, s, p, ceil, H, W, act = cfg
    torch.manual_seed(6)
    bn_a, bn_b = nn.BatchNorm2d(C).to(DEV), nn.BatchNorm2d(C).to(DEV)
    bn_a.weight.data.uniform_(0.5, 1.5)
    bn_a.bias.data.uniform_(-0.3, 0.3)
    bn_b.load_state_dict(bn_a.state_dict())
    pool = nn.MaxPool2d(k, s, p, ceil_mode=ceil)
    x = _nhwc(torch.randn(8, C, H, W, device=DEV))
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    slope = 0.1 if act == "leaky" else 0.0
    ya = F.batch_norm_act_maxpool(xa, bn_a, act, slope, pool)
    yb = F.max_pool2d(F.batch_norm_act(xb, bn_b, act, slope), k, s, p, ceil)
    assert ya.shape == yb.shape
    _same_up_to_stat_rounding(ya, yb)
    dy = _nhwc(torch.randn(ya.shape, device=DEV))
    ya.backward(dy)
    yb.backward(dy)
    assert _rel(xa.grad, xb.grad) < 2e-2 and _cos(xa.grad, xb.grad) > 0.9999
    assert _rel(bn_a.weight.grad, bn_b.weight.grad) < 2e-3
    assert _rel(bn_a.bias.grad, bn_b.bias.grad) < 2e-3


@pytest.mark.parametrize("cin,filters,H", [(256, 256, 32), (128, 256, 32)], ids=["identity", "projection"])
def test_hourglass_bottleneck_block(cin, filters, H):
    """Stacked Hourglass pre-activation bottleneck in training mode: the identity block sums x's
    two gradients (residual path dy + BN1's dx) inside BN1's backward apply pass (GradJoin input
    join); the projection block keeps the autograd sum."""
    from deep_vision_amd.models.hourglass import BottleneckBlock

    torch.manual_seed(3)
    blk = BottleneckBlock(cin, filters, downsample=cin != filters).to(DEV)
    for m in blk.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.3, 0.3)
    x32 = torch.randn(16, cin, H, H, device=DEV).bfloat16().float()
    _check_module(blk, x32)
