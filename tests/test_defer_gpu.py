"""Deferred BatchNorm applies (ops.defer, csrc/conv_fwd.hip AT_*): the BN elementwise passes of
the ResNet bottleneck folded into the A-operand load of the consuming 1x1 conv / dgrad.

The fused kernels compute exactly the fp32 expression of the standalone apply passes and feed
the MFMAs the same bf16 values the LDS-DMA path would load from the materialised tensor, so a
training step must be BITWISE identical with the deferral on and off (deterministic weight
gradients). Checked on ResNet-50 -- every deferral kind occurs in it: bn2 -> conv3 (AT_BN), the
identity and projection output joins -> next conv1 (AT_JOIN), bn3 -> conv3 dgrad with mask bits
(AT_BWDB, plain and after a projection join), bn1 -> conv1 dgrad with the mask from x (AT_BWDX,
stride-1 and strided scatter, with the lazy shortcut and the fused BN-backward sums)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _step(model, x, y):
    from deep_vision_amd import ops as F

    for p in model.parameters():
        p.grad = None
    out = model(x)
    loss = F.cross_entropy(out, y)
    loss.backward()
    torch.cuda.synchronize()
    return out.detach().float(), loss.item()


@pytest.mark.parametrize("hw", [64, 96])
def test_resnet50_step_bitwise_with_and_without_deferral(hw):
    from deep_vision_amd import set_deterministic
    from deep_vision_amd.models import ResNet50
    from deep_vision_amd.ops import defer

    set_deterministic(True)
    try:
        torch.manual_seed(0)
        base = ResNet50().to(DEV)
        x = torch.randn(8, 3, hw, hw, device=DEV)
        y = torch.randint(0, 1000, (8,), device=DEV)
        res = {}
        for on in (False, True):
            m = copy.deepcopy(base)
            defer.ENABLED = on
            for k in defer.COUNTERS:
                defer.COUNTERS[k] = 0
            outs = [_step(m, x, y) for _ in range(2)]  # 2 steps: BN shifts / running stats move
            grads = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
            bufs = {n: b.detach().clone() for n, b in m.named_buffers()}
            res[on] = (outs, grads, bufs, dict(defer.COUNTERS))
    finally:
        defer.ENABLED = True
        set_deterministic(False)
    (o0, g0, b0, c0), (o1, g1, b1, c1) = res[False], res[True]
    assert c0["fwd_fused"] == 0 and c0["bwd_fused"] == 0
    # per step: 16 bn2->conv3 + 12 joins (3+4+6+3 blocks minus the 4 stage-final ones) forward;
    # 16 bn3 -> conv3 dgrad + 16 bn1 -> conv1 dgrad backward (minus any that had to materialise)
    assert c1["fwd_fused"] == 2 * 28, c1
    assert c1["bwd_fused"] >= 2 * 28, c1
    assert c1["fwd_materialized"] == 0, c1
    for (a, la), (b, lb) in zip(o0, o1):
        assert la == lb
        assert torch.equal(a, b)
    for n in g0:
        assert torch.equal(g0[n], g1[n]), n
    for n in b0:
        assert torch.equal(b0[n], b1[n]), n


def test_pending_output_resolved_for_foreign_consumer():
    """A deferred output read by a consumer that cannot fold it (a 3x3 conv) is materialised first."""
    from deep_vision_amd import nn, ops as F
    from deep_vision_amd.ops import defer

    torch.manual_seed(1)
    conv = nn.Conv2d(64, 64, 3, padding=1, bias=False).to(DEV)
    bn = nn.BatchNorm2d(64).to(DEV)
    nxt = nn.Conv2d(64, 64, 3, padding=1, bias=False).to(DEV)
    x = torch.randn(4, 64, 16, 16, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    bn0 = copy.deepcopy(bn)
    a = F.conv_bn_act(x, conv, bn, "relu", defer_out=True)
    assert defer.pending(a) is not None
    ya = F.conv2d(a, nxt.weight, None, 1, 1)
    assert defer.pending(a) is None
    bn2 = copy.deepcopy(bn0)
    defer.ENABLED = False
    try:
        b = F.conv_bn_act(x, conv, bn2, "relu", defer_out=True)
        yb = F.conv2d(b, nxt.weight, None, 1, 1)
    finally:
        defer.ENABLED = True
    torch.cuda.synchronize()
    assert torch.equal(a, b) and torch.equal(ya, yb)
