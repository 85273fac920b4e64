"""BatchNorm batch statistics with a large mean.

Single-pass E[x^2] - mean^2 over fp32 partial sums cancels once |mean| >> std. The producers now
sum d = x - K and d^2 with K = the BN's previous batch mean (csrc/kernels.h DV_STAT_ROWS), so from
the second step on the variance is computed from centred data. Checked against fp64 statistics of
exactly the values the kernel sees, for the three producers: the unfused statistics pass (bf16
input), the conv epilogue (fp32 accumulators) and the depthwise epilogue. momentum = 1 makes
running_mean / running_var the batch mean / unbiased batch variance.
"""
import pytest
import torch
import torch.nn.functional as TF

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _nhwc(t):
    return t.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


def _check(bn, ref, step, offset):
    mean, var = ref.mean((0, 2, 3)), ref.var((0, 2, 3), unbiased=True)
    em = ((bn.running_mean.double() - mean).abs() / var.sqrt()).max().item()
    ev = ((bn.running_var.double() - var).abs() / var).max().item()
    # step 0 runs unshifted (K = 0): allow the cancellation error of E[x^2] - mean^2 there
    tol_v = 1e-3 if step > 0 else max(1e-3, 5e-6 * offset ** 2)
    assert em < 1e-3, (step, em)
    assert ev < tol_v, (step, ev)


@pytest.mark.parametrize("offset", [0.0, 30.0, 100.0])
def test_unfused_bn_stats_offset(offset):
    from deep_vision_amd import nn

    torch.manual_seed(1)
    C = 64
    bn = nn.BatchNorm2d(C, momentum=1.0).to(DEV)
    base = (1 + torch.rand(C, device=DEV))[None, :, None, None]  # per-channel means in [offset, 2 offset]
    for step in range(3):
        mu = offset * (1 + 0.05 * step) * base  # the batch mean drifts 5 % per step
        x = _nhwc(mu + torch.randn(8, C, 12, 12, device=DEV))
        y = bn(x)
        torch.cuda.synchronize()
        _check(bn, x.double(), step, offset)
        z = (x.double() - bn.running_mean.double()[None, :, None, None]) / (
            bn.running_var.double()[None, :, None, None] * (8 * 144 - 1) / (8 * 144) + bn.eps).sqrt()
        assert (y.double() - z).abs().max().item() < 5e-2


@pytest.mark.parametrize("offset", [0.0, 30.0, 100.0])
def test_conv_epilogue_stats_offset(offset):
    from deep_vision_amd import nn, ops as F

    torch.manual_seed(2)
    conv = nn.Conv2d(64, 128, 1, bias=False).to(DEV)
    bn = nn.BatchNorm2d(128, momentum=1.0).to(DEV)
    with torch.no_grad():  # positive weights: the output mean ~ offset, its std ~ 1
        conv.weight.copy_((torch.rand(128, 64, 1, 1, device=DEV) + 0.5) / 64)
    wq = conv.weight.detach().bfloat16().float()
    for step in range(3):
        x32 = (offset * (1 + 0.05 * step) + 8 * torch.randn(8, 64, 14, 14, device=DEV)).bfloat16().float()
        F.conv_bn_act(_nhwc(x32), conv, bn, "relu")
        torch.cuda.synchronize()
        ref = TF.conv2d(x32.double(), wq.double())
        _check(bn, ref, step, offset)


@pytest.mark.parametrize("offset", [0.0, 100.0])
def test_depthwise_epilogue_stats_offset(offset):
    from deep_vision_amd import ops as F
    from deep_vision_amd.ops.conv import STAT_ROWS

    torch.manual_seed(3)
    C = 128
    w = (torch.rand(C, 1, 3, 3, device=DEV) + 0.5) / 9
    wq = w.bfloat16().float()
    stats = torch.zeros(STAT_ROWS, C, device=DEV)
    for step in range(3):
        x32 = (offset + 3 * torch.randn(4, C, 14, 14, device=DEV)).bfloat16().float()
        y, st = F.conv2d(_nhwc(x32), w, None, 1, 1, 1, C, want_stats=True, stats_buf=stats)
        ref = TF.conv2d(x32.double(), w.double(), None, 1, 1, 1, C)
        # fold the shards the way bn_finalize does: mean = K + E[d], var = E[d^2] - E[d]^2
        n = ref.numel() // C
        k = st[128].double()
        sh = st[:128].reshape(64, 2, C).double().sum(0)
        mean, var = k + sh[0] / n, sh[1] / n - (sh[0] / n) ** 2
        rm, rv = ref.mean((0, 2, 3)), ref.var((0, 2, 3), unbiased=False)
        assert ((mean - rm).abs() / rv.sqrt()).max() < 1e-3
        tol = 2e-3 if step > 0 else max(2e-3, 5e-6 * offset ** 2)
        assert ((var - rv).abs() / rv).max() < tol
        # emulate the finalize: re-zero the shards, next shift = this batch mean
        st[:128].zero_()
        st[128].copy_(mean.float())


def test_nonfinite_batch_does_not_poison_shift():
    """the finalize stores each batch mean as the next batch's shift. A batch with an
    Inf/NaN must not leave a non-finite shift behind: the following finite batch's statistics
    (and so training after a skipped step) must be exact again."""
    from deep_vision_amd import nn

    torch.manual_seed(3)
    C = 64
    bn = nn.BatchNorm2d(C, momentum=1.0).to(DEV)
    bad = torch.randn(8, C, 12, 12, device=DEV)
    bad[0, 3, 0, 0] = float("inf")
    bad[1, 7, 2, 2] = float("nan")
    bn(_nhwc(bad))
    torch.cuda.synchronize()
    x = _nhwc(5 + torch.randn(8, C, 12, 12, device=DEV))
    y = bn(x)
    torch.cuda.synchronize()
    assert torch.isfinite(bn.running_mean).all() and torch.isfinite(bn.running_var).all()
    assert torch.isfinite(y.float()).all()
    _check(bn, x.double(), 1, 5.0)
