"""Grouped 1x1 convolution with a fused channel shuffle (csrc/gconv.hip; SURVEY §2.7 K7, VERDICT r2
next #7) against plain PyTorch fp32 (conv2d(groups) + the ShuffleNet channel shuffle): output,
BatchNorm partial statistics, input and weight gradients, at g = 3 with 20 / 40 / 80 channels per
group, the dense (g = 1) conv followed by a 3-group shuffle, and a whole ShuffleNet V1 unit."""
import pytest
import torch
import torch.nn.functional as TF

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6)).item()


def _nhwc(t):
    return t.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


def _shuffle(y, g):
    N, C, H, W = y.shape
    return y.reshape(N, g, C // g, H, W).transpose(1, 2).reshape(N, C, H, W)


@pytest.mark.parametrize("G,Cg,Og", [(3, 20, 80), (3, 80, 20), (3, 40, 40), (3, 20, 72), (1, 24, 60), (3, 80, 160)])
@pytest.mark.parametrize("shuffle", [0, 3])
def test_gconv_fwd_bwd_stats(G, Cg, Og, shuffle):
    from deep_vision_amd import ops as F
    from deep_vision_amd.ops.conv import STAT_ROWS

    torch.manual_seed(G * 1000 + Cg + Og)
    N, H, W = 3, 9, 11  # M = 297: a partial row tile
    C, O = G * Cg, G * Og
    x32 = torch.randn(N, C, H, W, device=DEV).bfloat16().float()
    w = (torch.randn(O, Cg, 1, 1, device=DEV) * Cg ** -0.5).requires_grad_(True)
    x = _nhwc(x32).requires_grad_(True)
    stats = torch.zeros(STAT_ROWS, O, device=DEV)
    y, st = F.conv2d(x, w, None, 1, 0, 1, G, want_stats=True, stats_buf=stats, shuffle=shuffle)
    assert st is not None and st.data_ptr() == stats.data_ptr()
    xr = x32.clone().requires_grad_(True)
    wr = w.detach().bfloat16().float().requires_grad_(True)
    yr = TF.conv2d(xr, wr, None, 1, 0, 1, G)
    if shuffle:
        yr = _shuffle(yr, shuffle)
    assert y.shape == yr.shape
    assert _rel(y, yr) < 1e-2
    # statistics by stored channel (fresh buffer: zero shift), of the fp32 results
    tot = st[:128].reshape(64, 2, O).double().sum(0)
    yd = yr.detach().double()
    assert _rel(tot[0], yd.sum((0, 2, 3))) < 1e-3
    assert _rel(tot[1], (yd * yd).sum((0, 2, 3))) < 1e-3
    dy32 = torch.randn_like(yr).bfloat16().float()
    y.backward(_nhwc(dy32))
    yr.backward(dy32)
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(w.grad, wr.grad) < 2e-2


def test_shufflenet_unit_native_vs_torch():
    from deep_vision_amd.models.mobilenet import ShuffleUnit
    from deep_vision_amd.ops.common import set_backend

    torch.manual_seed(0)
    for cin, cout, stride in ((240, 240, 1), (240, 480, 2)):
        u = ShuffleUnit(cin, cout, 3, stride).to(DEV).train()
        ref = ShuffleUnit(cin, cout, 3, stride).to(DEV).train()
        ref.load_state_dict(u.state_dict())
        x32 = torch.randn(8, cin, 14, 14, device=DEV).bfloat16().float()
        x = _nhwc(x32).requires_grad_(True)
        y = u(x)
        set_backend("torch")
        try:
            xr = x32.clone().requires_grad_(True)
            yr = ref(xr)
        finally:
            set_backend("native")
        cos = TF.cosine_similarity(y.float().flatten(), yr.float().flatten(), 0).item()
        assert cos > 0.999, cos
        g = torch.randn_like(yr)
        y.backward(_nhwc(g))
        yr.backward(g)
        assert TF.cosine_similarity(x.grad.float().flatten(), xr.grad.float().flatten(), 0).item() > 0.995
        named = dict(ref.named_parameters())
        for (n, a), b in zip(u.named_parameters(), ref.parameters()):
            # bn1.weight / bn2.bias have an exactly-zero true gradient (the depthwise conv -> bn2
            # chain is invariant to them, tests/test_concat_gpu.py): both backends return rounding
            # noise there -- it must be small next to the sibling parameter's gradient
            sib = named.get(n.rsplit(".", 1)[0] + (".bias" if n.endswith("weight") else ".weight"))
            if sib is not None and b.grad.norm() < 1e-3 * sib.grad.norm():
                assert a.grad.norm() < 2e-2 * sib.grad.norm(), n
                continue
            c = TF.cosine_similarity(a.grad.float().flatten(), b.grad.float().flatten(), 0).item()
            assert c > 0.99, (n, c)
